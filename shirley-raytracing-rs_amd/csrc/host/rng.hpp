// rng.hpp — seeded replacement for the reference's rand::thread_rng() in scene construction.
//
// The reference builds scenes and Perlin tables from thread_rng (scenes.rs:137, perlin/mod.rs:74),
// which cannot be seeded.  This host draws them from Philox4x32-10 streams keyed by the scene seed:
// counter = (n/2 low, n/2 high, 0xFFFFFFFF, stream) with stream >= 1, disjoint from the per-path
// render streams (counter word 3 == 0, see trace.hip).
#pragma once

#include <cmath>
#include <cstdint>
#include <vector>

namespace host {

enum : uint32_t {
  kStreamRandomScene = 1,  // random_scene (scenes.rs:281-429)
  kStreamGenSpheres = 2,   // gen_spheres (benches/my_benchmark.rs:35-60)
  kStreamFinalScene = 3,   // book-2 final_scene (extension; absent from the reference)
  kStreamPerlinBase = 16   // Perlin table j (perlin/mod.rs:73-85) uses stream 16 + j
};

inline void philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1) {
  for (int r = 0; r < 10; ++r) {
    if (r) {
      k0 += 0x9E3779B9u;
      k1 += 0xBB67AE85u;
    }
    uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
    uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
    uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0;
    uint32_t n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
    c[1] = (uint32_t)p1;
    c[3] = (uint32_t)p0;
    c[0] = n0;
    c[2] = n2;
  }
}

class SceneRng {
 public:
  SceneRng(uint64_t seed, uint32_t stream) : seed_(seed), stream_(stream) {}

  uint64_t next_u64() {
    uint32_t c[4] = {(uint32_t)(n_ >> 1), (uint32_t)(n_ >> 33), 0xFFFFFFFFu, stream_};
    philox4x32_10(c, (uint32_t)seed_, (uint32_t)(seed_ >> 32));
    uint64_t v = (n_ & 1) ? ((uint64_t)c[2] | ((uint64_t)c[3] << 32)) : ((uint64_t)c[0] | ((uint64_t)c[1] << 32));
    ++n_;
    return v;
  }
  // rng.gen::<f64>() (rand 0.8 Standard): 53 random bits in [0, 1)
  double gen_f64() { return (double)(next_u64() >> 11) * (1.0 / 9007199254740992.0); }
  // core/math.rs:22-25 random_real
  double random_real(double mn, double mx) { return mn + (mx - mn) * gen_f64(); }
  // rng.gen_range(0..n): unbiased (Lemire's widening multiply with rejection)
  uint64_t gen_range(uint64_t n) {
    uint64_t x = next_u64();
    unsigned __int128 m = (unsigned __int128)x * n;
    uint64_t l = (uint64_t)m;
    if (l < n) {
      uint64_t t = (0 - n) % n;
      while (l < t) {
        x = next_u64();
        m = (unsigned __int128)x * n;
        l = (uint64_t)m;
      }
    }
    return (uint64_t)(m >> 64);
  }
  // SliceRandom::choose_weighted (rand 0.8 WeightedIndex): uniform in [0, total), then the number of
  // cumulative weights (all but the last) that are <= the draw.
  size_t choose_weighted(const std::vector<double>& w) {
    std::vector<double> cum;
    double total = 0.0;
    for (size_t i = 0; i < w.size(); ++i) {
      total += w[i];
      if (i + 1 < w.size()) cum.push_back(total);
    }
    double x = total * gen_f64();
    size_t k = 0;
    while (k < cum.size() && cum[k] <= x) ++k;
    return k;
  }
  // standard normal (Box-Muller); rand_distr uses a Ziggurat — same distribution, different stream
  double gen_normal() {
    double u1 = gen_f64(), u2 = gen_f64();
    if (u1 <= 0.0) u1 = 1.0 / 9007199254740992.0;
    return std::sqrt(-2.0 * std::log(u1)) * std::cos(2.0 * 3.14159265358979323846 * u2);
  }

 private:
  uint64_t seed_;
  uint32_t stream_;
  uint64_t n_ = 0;
};

}  // namespace host
