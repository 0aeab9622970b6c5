// keycheck_sim — drives rt_render_sharded's cross-rank agreement rule (csrc/rt/keycheck.h) for a sequence
// of calls on `world` simulated ranks, so tests/test_keycheck.py checks its decisions on the CPU.
//   keycheck_sim <world> <strict 0|1> <call> [<call> ...]
// a call is one comma-separated (digest:key) or (key) per rank, hexadecimal (digest defaults to 1).
// Prints one line per call, one token per rank:
//   S  checked in the call, agreed; frame collectives issued
//   A  key unchanged: check deferred to the next call; frame collectives issued
//   F<r><w>  check in the call failed (first differing rank r, w = s scene / k key): no frame collectives
//   P<r><w>  the deferred check of the previous call failed: no gather, no frame collectives
// followed by " gather=same" when every rank issued this call's all-gather, else " gather=diverged".
// The simulation mirrors check_call_key in rt_api.cpp: deferred check, then the gather, then the
// immediate check when key_check_now says so.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../shirley-raytracing-rs_amd/csrc/rt/keycheck.h"

int main(int argc, char** argv) {
  if (argc < 4) {
    std::fprintf(stderr, "usage: %s <world> <strict> <call> [...]\n", argv[0]);
    return 2;
  }
  const int world = std::atoi(argv[1]);
  const bool strict = std::atoi(argv[2]) != 0;
  std::vector<rt::KeyState> ks(world);
  std::vector<std::vector<uint64_t>> pending_words(world);  // the words each rank's deferred check reads
  for (int a = 3; a < argc; ++a) {
    std::vector<uint64_t> digest(world, 1), key(world, 0);
    std::string s = argv[a];
    size_t pos = 0;
    for (int r = 0; r < world; ++r) {
      size_t end = s.find(',', pos);
      std::string tok = s.substr(pos, end == std::string::npos ? std::string::npos : end - pos);
      size_t colon = tok.find(':');
      if (colon != std::string::npos) {
        digest[r] = std::strtoull(tok.substr(0, colon).c_str(), nullptr, 16);
        key[r] = std::strtoull(tok.substr(colon + 1).c_str(), nullptr, 16);
      } else {
        key[r] = std::strtoull(tok.c_str(), nullptr, 16);
      }
      pos = end == std::string::npos ? s.size() : end + 1;
    }
    // phase 1: each rank's deferred check of its previous call
    std::vector<std::string> out(world);
    std::vector<bool> gathers(world, true);
    for (int r = 0; r < world; ++r) {
      if (!ks[r].pending) continue;
      ks[r].pending = false;
      int what = 0;
      const int bad = rt::key_mismatch(pending_words[r].data(), world, &what);
      if (bad >= 0) {
        ks[r].verified = false;
        out[r] = "P" + std::to_string(bad) + (what ? "k" : "s");
        gathers[r] = false;
      }
    }
    // phase 2: the call's all-gather (every rank still in the call) and the immediate or deferred check
    std::vector<uint64_t> words(2 * (size_t)world);
    for (int r = 0; r < world; ++r) {
      words[2 * r] = digest[r];
      words[2 * r + 1] = key[r];
    }
    bool all = true;
    for (int r = 0; r < world; ++r) all = all && gathers[r];
    for (int r = 0; r < world; ++r) {
      if (!gathers[r]) continue;
      if (rt::key_check_now(ks[r], key[r], strict)) {
        int what = 0;
        const int bad = rt::key_mismatch(words.data(), world, &what);
        if (bad >= 0) {
          ks[r].verified = false;
          out[r] = "F" + std::to_string(bad) + (what ? "k" : "s");
        } else {
          ks[r].verified = true;
          ks[r].verified_key = key[r];
          out[r] = "S";
        }
      } else {
        ks[r].pending = true;
        pending_words[r] = words;
        out[r] = "A";
      }
    }
    for (int r = 0; r < world; ++r) std::printf("%s%s", r ? " " : "", out[r].c_str());
    std::printf(" gather=%s\n", all ? "same" : "diverged");
  }
  return 0;
}
