// plan_check — prints rt::plan_samples (csrc/rt/plan.h: unit length, sample passes, scratch) for the
// calls given on the command line, so tests/test_plan.py checks the planning rules on the CPU.
//   plan_check <n_pix> <count> <engine> <lanes> <sample_chunk> <budget_bytes> [...6 more per call]
// prints one line per call: chunk n_chunks per_pass passes partial_bytes segments ok queue_window
#include <cstdio>
#include <cstdlib>

#include "../shirley-raytracing-rs_amd/csrc/rt/plan.h"

int main(int argc, char** argv) {
  if (argc < 7 || (argc - 1) % 6 != 0) {
    std::fprintf(stderr, "usage: %s <n_pix> <count> <engine> <lanes> <sample_chunk> <budget_bytes> ...\n", argv[0]);
    return 2;
  }
  for (int i = 1; i + 5 < argc; i += 6) {
    const rt::SamplePlan P = rt::plan_samples(std::atoll(argv[i]), std::atoi(argv[i + 1]), std::atoi(argv[i + 2]),
                                              std::atoll(argv[i + 3]), std::atoi(argv[i + 4]), std::atoll(argv[i + 5]));
    std::printf("%d %d %d %d %lld %d %d %u\n", P.chunk, P.n_chunks, P.per_pass, P.passes, P.partial_bytes,
                P.segments ? 1 : 0, P.ok ? 1 : 0, P.queue_window);
  }
  return 0;
}
