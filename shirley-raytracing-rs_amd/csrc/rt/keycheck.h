// keycheck.h — the cross-rank agreement rule of rt_render_sharded (host only, pure: no HIP, no RCCL), so
// the decisions can be driven on the CPU (tests/test_keycheck.py through tools/keycheck_sim.cpp).
//
// Every rank must render the same scene with the same call key (scene digest + resolved partition, sample
// range and render arguments, rt_api.cpp call_key).  Every call, on every rank, all-gathers the 16-byte
// (digest, key) words — so all ranks issue one and the same collective sequence whatever their arguments —
// and the gathered words are checked on the host:
//   * now (before the frame's collectives are issued) when this rank's key differs from the one the ranks
//     last agreed on, or on every call in strict mode (SHIRLEY_KEY_CHECK=sync);
//   * otherwise at the rank's next call (deferred: a steady loop of frames needs no host round trip).
// All ranks read the same gathered words, so a check fails on every rank that performs it.  A correct
// program changes scene or arguments on every rank in the same call: every rank checks now and all fail
// together, before any frame collective.  The misuse — one rank changing its key alone — fails that rank
// now; its peers, whose keys did not change, have already issued the frame's collectives, which the failed
// rank never joins, so their stream waits there (they fail at their next call's deferred check, if their
// host gets there).  Strict mode makes every rank fail in the call itself, at one host round trip per call.
// A failed check (now or deferred) poisons the rank's communicator: its peers may still hold the failed
// call's frame collectives on it, and a later all-gather from this rank would be paired with them
// (mismatched types and sizes: undefined behaviour, not a stall).  So every later call on a poisoned
// communicator fails at once and issues nothing; the program destroys and re-creates it.
#pragma once

#include <stdint.h>

namespace rt {

struct KeyState {
  bool verified = false;      // the ranks agreed on verified_key at some call
  uint64_t verified_key = 0;
  bool pending = false;       // the previous call's gathered words are still to be checked
  bool poisoned = false;      // a check failed: no further collective on this communicator
};

// Whether a call must check its own gathered words before issuing the frame's collectives.
inline bool key_check_now(const KeyState& s, uint64_t key, bool strict) {
  return strict || !s.verified || s.verified_key != key;
}

// Gathered words [world][2] = (scene digest, call key) per rank.  Returns -1 when every rank agrees with
// rank 0, else the first rank that differs, with *what = 0 (scene digest) or 1 (call key).
inline int key_mismatch(const uint64_t* words, int world, int* what) {
  for (int r = 0; r < world; ++r)
    if (words[2 * r] != words[0]) {
      *what = 0;
      return r;
    }
  for (int r = 0; r < world; ++r)
    if (words[2 * r + 1] != words[1]) {
      *what = 1;
      return r;
    }
  return -1;
}

}  // namespace rt
