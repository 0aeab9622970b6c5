// Issue cost of the VALU instructions the trace kernel leans on (gfx950), measured with s_memtime:
// one wave per SIMD (4 waves per CU, all CUs), 8 independent chains per lane, N iterations.
// Prints shader cycles per wave-instruction.  Diagnostic only.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CHAINS 8
template <int OP>
__global__ __launch_bounds__(1024) void kern(int n, unsigned long long* out, unsigned* sink) {
  unsigned a[CHAINS];
  double f[CHAINS];
  unsigned long long w[CHAINS];
  for (int i = 0; i < CHAINS; ++i) {
    a[i] = threadIdx.x * 7919u + i;
    f[i] = 1.0 + 1e-3 * (threadIdx.x + i);
    w[i] = a[i];
  }
  unsigned k = 0xD2511F53u;
  unsigned long long sm = 0x5555aaaa3333ccccull ^ (unsigned long long)n;
  unsigned long long cm[CHAINS];
  for (int i = 0; i < CHAINS; ++i) cm[i] = sm >> i;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < n; ++it) {
#pragma unroll
    for (int i = 0; i < CHAINS; ++i) {
      if (OP == 0) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, 0" : "=v"(w[i]) : "v"(a[i]), "s"(k) : "vcc");
      if (OP == 1) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[i]) : "s"(k));
      if (OP == 2) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a[i]) : "s"(k));
      if (OP == 3) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a[i]) : "s"(k));
      if (OP == 4) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a[i]) : "s"(k));
      if (OP == 5) asm volatile("v_fma_f64 %0, %0, %0, 1.0" : "+v"(f[i]));
      if (OP == 6) asm volatile("v_add_f64 %0, %0, 1.0" : "+v"(f[i]));
      if (OP == 7) asm volatile("v_rcp_f64 %0, %0" : "+v"(f[i]));
      if (OP == 8) asm volatile("v_sqrt_f64 %0, %0" : "+v"(f[i]));
      if (OP == 9) asm volatile("v_fma_f32 %0, %0, %0, 1.0" : "+v"(a[i]));
      if (OP == 10) asm volatile("v_pk_fma_f32 %0, %0, %0, %0" : "+v"(w[i]));
      if (OP == 11) asm volatile("v_div_scale_f64 %0, vcc, %0, %0, 1.0" : "+v"(f[i]) : : "vcc");
      if (OP == 12) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a[i]) : "v"(a[(i + 1) % CHAINS]));
      if (OP == 13) asm volatile("v_cvt_f64_u32 %0, %1" : "=v"(f[i]) : "v"(a[i]));
      if (OP == 14) asm volatile("v_ldexp_f64 %0, %0, 1" : "+v"(f[i]));
      if (OP == 15) asm volatile("v_readlane_b32 %0, %1, 5" : "=s"(k) : "v"(a[i]));
      if (OP == 16) asm volatile("v_min_f64 %0, %0, %0" : "+v"(f[i]));
      if (OP == 17) asm volatile("v_cmp_lt_f64 vcc, %0, %1" : : "v"(f[i]), "v"(f[(i + 1) % CHAINS]) : "vcc");
      if (OP == 18) asm volatile("ds_bpermute_b32 %0, %1, %0\n s_waitcnt lgkmcnt(0)" : "+v"(a[i]) : "v"(a[(i + 3) % CHAINS]));
      if (OP == 19) asm volatile("v_mad_u32_u24 %0, %0, %1, %0" : "+v"(a[i]) : "s"(k));
      if (OP == 20) asm volatile("v_mul_f64 %0, %0, %0" : "+v"(f[i]));
      if (OP == 21) asm volatile("v_cvt_f32_f64 %0, %1" : "=v"(a[i]) : "v"(f[i]));
      if (OP == 22) asm volatile("v_mov_b64 %0, %1" : "=v"(w[i]) : "v"(f[(i + 1) % CHAINS]));
      if (OP == 23) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(a[i]) : "v"(a[(i + 1) % CHAINS]), "s"(k));
      if (OP == 24) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(a[(i + 1) % CHAINS]), "s"(k));
      if (OP == 25) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[i]) : "s"(k));
      if (OP == 26) asm volatile("v_mov_b32_dpp %0, %1 row_shr:1" : "=v"(a[i]) : "v"(a[(i + 1) % CHAINS]));
      if (OP == 27) asm volatile("v_cndmask_b32 %0, %0, %1, vcc\n v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a[i]) : "v"(a[(i + 1) % CHAINS]));
      if (OP == 28) asm volatile("v_max3_f32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(a[(i + 1) % CHAINS]), "s"(k));
      if (OP == 29) asm volatile("v_lshl_add_u64 %0, %0, 3, %1" : "+v"(w[i]) : "v"(w[(i + 1) % CHAINS]));
      if (OP == 30) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(a[i]) : "v"(k), "s"(sm));
      if (OP == 31) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a[i]) : "v"(k) : );
      if (OP == 32) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(a[i]) : "v"(a[(i + 1) % CHAINS]), "s"(sm));
      if (OP == 33) asm volatile("v_cmp_lt_u32 %0, %1, %2" : "=s"(cm[i]) : "v"(a[i]), "v"(k));
      if (OP == 34) asm volatile("v_cmp_lt_u32 vcc, %0, %1\n v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a[i]) : "v"(k) : "vcc");
      if (OP == 35) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(a[i]) : "v"(k), "s"(cm[i]));
      if (OP == 36) asm volatile("v_max_u32 %0, %0, %1" : "+v"(a[i]) : "v"(a[(i + 1) % CHAINS]));
      // lane-mask reads: VCC written by a compare right before / two selects on one compare / a stale VCC
      // read through the VOP3 form / a compare into an SGPR pair then a VOP3 select
      if (OP == 37) asm volatile("v_cmp_lt_u32 vcc, %0, %1\n v_cndmask_b32 %0, %0, %1, vcc\n v_cndmask_b32 %1, %1, %0, vcc" : "+v"(a[i]), "+v"(a[(i + 1) % CHAINS]) : : "vcc");
      if (OP == 38) asm volatile("v_cndmask_b32_e64 %0, %0, %1, vcc" : "+v"(a[i]) : "v"(a[(i + 1) % CHAINS]));
      if (OP == 39) asm volatile("v_cmp_lt_u32_e64 %2, %0, %1\n s_nop 1\n v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(a[i]) : "v"(k), "s"(cm[i]));
      if (OP == 40) asm volatile("s_mov_b64 vcc, %1\n v_cndmask_b32 %0, %0, %0, vcc" : "+v"(a[i]) : "s"(sm) : "vcc");
      if (OP == 41) asm volatile("v_cmp_lt_u32 vcc, %0, %1\n v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a[i]) : "v"(k) : "vcc");
      if (OP == 42) asm volatile("v_cmp_lt_f32 vcc, %0, %1\n v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a[i]) : "v"(k) : "vcc");
      // the leaf tests' pattern: two compares combined by SALU, then two selects (VOP2 vs VOP3 form)
      if (OP == 43) asm volatile("v_cmp_lt_u32 vcc, %0, %3\n v_cmp_gt_u32_e64 %2, %1, %3\n s_and_b64 vcc, vcc, %2\n v_cndmask_b32 %0, %0, %3, vcc\n v_cndmask_b32 %1, %1, %3, vcc" : "+v"(a[i]), "+v"(a[(i + 1) % CHAINS]), "=&s"(cm[i]) : "v"(k) : "vcc");
      if (OP == 44) asm volatile("v_cmp_lt_u32 vcc, %0, %3\n v_cmp_gt_u32_e64 %2, %1, %3\n s_and_b64 vcc, vcc, %2\n v_cndmask_b32_e64 %0, %0, %3, vcc\n v_cndmask_b32_e64 %1, %1, %3, vcc" : "+v"(a[i]), "+v"(a[(i + 1) % CHAINS]), "=&s"(cm[i]) : "v"(k) : "vcc");
      if (OP == 45) asm volatile("v_cmp_lt_u32 vcc, %0, %3\n v_cmp_gt_u32_e64 %2, %1, %3\n s_and_b64 %2, vcc, %2\n v_cndmask_b32_e64 %0, %0, %3, %2\n v_cndmask_b32_e64 %1, %1, %3, %2" : "+v"(a[i]), "+v"(a[(i + 1) % CHAINS]), "=&s"(cm[i]) : "v"(k) : "vcc");
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  unsigned s = 0;
  for (int i = 0; i < CHAINS; ++i) s ^= (unsigned)cm[i];
  for (int i = 0; i < CHAINS; ++i) s ^= a[i] ^ (unsigned)w[i] ^ (unsigned)(w[i] >> 32) ^ (unsigned)__double_as_longlong(f[i]);
  if (s == 0x12345678u) sink[0] = s;
  if (threadIdx.x % 64 == 0) out[blockIdx.x * 12 + threadIdx.x / 64] = t1 - t0;
}

static int g_threads = 256;
template <int OP>
double run(int n, int blocks, unsigned long long* d, unsigned* sink) {
  hipLaunchKernelGGL(kern<OP>, dim3(blocks), dim3(g_threads), 0, 0, n, d, sink);
  hipLaunchKernelGGL(kern<OP>, dim3(blocks), dim3(g_threads), 0, 0, n, d, sink);
  (void)hipDeviceSynchronize();
  static unsigned long long h[4096 * 3];
  const int waves = blocks * g_threads / 64;
  (void)hipMemcpy(h, d, blocks * 12 * 8, hipMemcpyDeviceToHost);
  double s = 0;
  int cnt = 0;
  for (int b = 0; b < blocks; ++b)
    for (int w = 0; w < g_threads / 64; ++w) { s += (double)h[b * 12 + w]; ++cnt; }
  (void)waves;
  // per-SIMD issue cost: per-wave time / (waves per SIMD)
  return s / cnt / ((double)n * CHAINS) / (g_threads / 256.0);
}

int main(int argc, char** argv) {
  const int n = 4096, blocks = 256;
  g_threads = argc > 1 ? atoi(argv[1]) : 256;
  unsigned long long* d;
  unsigned* sink;
  (void)hipMalloc(&d, 4096 * 12 * 8);
  (void)hipMalloc(&sink, 4);
  const char* names[] = {"v_mad_u64_u32", "v_mul_lo_u32", "v_mul_hi_u32", "v_mul_u32_u24", "v_xor_b32",
                         "v_fma_f64", "v_add_f64", "v_rcp_f64", "v_sqrt_f64", "v_fma_f32", "v_pk_fma_f32",
                         "v_div_scale_f64", "v_cndmask_b32", "v_cvt_f64_u32", "v_ldexp_f64", "v_readlane_b32",
                         "v_min_f64", "v_cmp_lt_f64", "ds_bpermute+wait", "v_mad_u32_u24", "v_mul_f64",
                         "v_cvt_f32_f64", "v_mov_b64", "v_bitop3_b32", "v_perm_b32", "v_add_u32", "v_mov_b32_dpp",
                         "2x v_cndmask_b32", "v_max3_f32", "v_lshl_add_u64", "cndmask_e64 s-mask", "cndmask vcc const",
                         "cndmask_e64 s nb", "v_cmp_lt_u32 ->s", "cmp+cndmask vcc", "cndmask_e64 cm", "v_max_u32 nb",
                         "cmp+2x cndmask vcc", "cndmask_e64 vcc", "cmp_e64+nop+cndmask", "s_mov vcc+cndmask",
                         "cmp,2 add,cndmask", "cmp_f32+cndmask", "2cmp,s_and vcc,2 cnd32", "2cmp,s_and vcc,2 cnd64",
                         "2cmp,s_and s,2 cnd64"};
  const int nops = 46;
  double c[46];
  c[0] = run<0>(n, blocks, d, sink); c[1] = run<1>(n, blocks, d, sink); c[2] = run<2>(n, blocks, d, sink);
  c[3] = run<3>(n, blocks, d, sink); c[4] = run<4>(n, blocks, d, sink); c[5] = run<5>(n, blocks, d, sink);
  c[6] = run<6>(n, blocks, d, sink); c[7] = run<7>(n, blocks, d, sink); c[8] = run<8>(n, blocks, d, sink);
  c[9] = run<9>(n, blocks, d, sink); c[10] = run<10>(n, blocks, d, sink); c[11] = run<11>(n, blocks, d, sink);
  c[12] = run<12>(n, blocks, d, sink); c[13] = run<13>(n, blocks, d, sink); c[14] = run<14>(n, blocks, d, sink);
  c[15] = run<15>(n, blocks, d, sink); c[16] = run<16>(n, blocks, d, sink); c[17] = run<17>(n, blocks, d, sink);
  c[18] = run<18>(n, blocks, d, sink); c[19] = run<19>(n, blocks, d, sink); c[20] = run<20>(n, blocks, d, sink);
  c[21] = run<21>(n, blocks, d, sink); c[22] = run<22>(n, blocks, d, sink); c[23] = run<23>(n, blocks, d, sink);
  c[24] = run<24>(n, blocks, d, sink); c[25] = run<25>(n, blocks, d, sink); c[26] = run<26>(n, blocks, d, sink);
  c[27] = run<27>(n, blocks, d, sink); c[28] = run<28>(n, blocks, d, sink); c[29] = run<29>(n, blocks, d, sink);
  c[30] = run<30>(n, blocks, d, sink); c[31] = run<31>(n, blocks, d, sink); c[32] = run<32>(n, blocks, d, sink);
  c[33] = run<33>(n, blocks, d, sink); c[34] = run<34>(n, blocks, d, sink); c[35] = run<35>(n, blocks, d, sink);
  c[36] = run<36>(n, blocks, d, sink); c[37] = run<37>(n, blocks, d, sink); c[38] = run<38>(n, blocks, d, sink);
  c[39] = run<39>(n, blocks, d, sink); c[40] = run<40>(n, blocks, d, sink); c[41] = run<41>(n, blocks, d, sink);
  c[42] = run<42>(n, blocks, d, sink); c[43] = run<43>(n, blocks, d, sink); c[44] = run<44>(n, blocks, d, sink);
  c[45] = run<45>(n, blocks, d, sink);
  printf("threads/block %d (%d waves per SIMD): SIMD cycles per wave-instruction\n", g_threads, g_threads / 256);
  for (int i = 0; i < nops; ++i) printf("%-18s %6.2f\n", names[i], c[i]);
  return 0;
}
