// keycheck_sim — drives rt_render_sharded's cross-rank agreement rule (csrc/rt/keycheck.h) for a sequence
// of calls on `world` simulated ranks, so tests/test_keycheck.py checks its decisions on the CPU.
//   keycheck_sim <world> <strict 0|1> <call> [<call> ...]
// a call is one comma-separated (digest:key) or (key) per rank, hexadecimal (digest defaults to 1).
// Prints one line per call, one token per rank:
//   S  checked in the call, agreed; frame collectives issued
//   A  key unchanged: check deferred to the next call; frame collectives issued
//   F<r><w>  check in the call failed (first differing rank r, w = s scene / k key): no frame collectives
//   P<r><w>  the deferred check of the previous call failed: no gather, no frame collectives
//   X  the communicator is poisoned by an earlier failed check: the call fails at once, issues nothing
// followed by " gather=same" when every rank issued this call's all-gather, else " gather=diverged", and
// " pairing=ok" while every rank's sequence of issued collectives (all-gathers G, frame collectives F) is a
// prefix of another's — RCCL then pairs like with like, and a rank that is behind only stalls its peers —,
// else " pairing=mismatch" (a G paired with an F: undefined).
// The simulation mirrors check_call_key and rt_render_sharded in rt_api.cpp: poisoned communicator, deferred
// check, then the gather, then the immediate check when key_check_now says so, then the frame.
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
  std::vector<std::string> issued(world);                    // collectives each rank issued, in order
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
      if (ks[r].poisoned) {
        out[r] = "X";
        gathers[r] = false;
        continue;
      }
      if (!ks[r].pending) continue;
      ks[r].pending = false;
      int what = 0;
      const int bad = rt::key_mismatch(pending_words[r].data(), world, &what);
      if (bad >= 0) {
        ks[r].verified = false;
        ks[r].poisoned = true;
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
      issued[r] += 'G';
      if (rt::key_check_now(ks[r], key[r], strict)) {
        int what = 0;
        const int bad = rt::key_mismatch(words.data(), world, &what);
        if (bad >= 0) {
          ks[r].verified = false;
          ks[r].poisoned = true;
          out[r] = "F" + std::to_string(bad) + (what ? "k" : "s");
        } else {
          ks[r].verified = true;
          ks[r].verified_key = key[r];
          out[r] = "S";
          issued[r] += 'F';
        }
      } else {
        ks[r].pending = true;
        pending_words[r] = words;
        out[r] = "A";
        issued[r] += 'F';
      }
    }
    bool pairing = true;
    for (int a = 0; a < world; ++a)
      for (int b = 0; b < world; ++b) {
        const std::string& x = issued[a].size() <= issued[b].size() ? issued[a] : issued[b];
        const std::string& y = issued[a].size() <= issued[b].size() ? issued[b] : issued[a];
        pairing = pairing && y.compare(0, x.size(), x) == 0;
      }
    for (int r = 0; r < world; ++r) std::printf("%s%s", r ? " " : "", out[r].c_str());
    std::printf(" gather=%s pairing=%s\n", all ? "same" : "diverged", pairing ? "ok" : "mismatch");
  }
  return 0;
}
