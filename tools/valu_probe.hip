// valu_probe.hip -- issue throughput of the integer VALU instructions the
// CityHash kernels are made of, on gfx950 (tools only, not product code).
//
// Every wave runs ITERS iterations of 8 independent chains of one
// instruction (inline asm, so the count is exact); W waves per SIMD run at
// once (one workgroup of 4W waves per CU, 256 CUs).  Each wave stamps
// s_memtime around its loop; cycles per instruction per SIMD =
// wave cycles / (instructions per wave * W).
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/bin/valu_probe tools/valu_probe.hip
//   tools/bin/valu_probe            -> one JSON line per (op, waves per SIMD)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

constexpr int ITERS = 2000;

#define CHAIN8(INSN)                                                                  \
  asm volatile(INSN : "+v"(a0) : "v"(b));                                             \
  asm volatile(INSN : "+v"(a1) : "v"(b));                                             \
  asm volatile(INSN : "+v"(a2) : "v"(b));                                             \
  asm volatile(INSN : "+v"(a3) : "v"(b));                                             \
  asm volatile(INSN : "+v"(a4) : "v"(b));                                             \
  asm volatile(INSN : "+v"(a5) : "v"(b));                                             \
  asm volatile(INSN : "+v"(a6) : "v"(b));                                             \
  asm volatile(INSN : "+v"(a7) : "v"(b));

template <int OP>
__global__ __launch_bounds__(1024) void k_probe(unsigned long long *cyc, unsigned *sink, unsigned seed) {
  typedef unsigned long long u64;
  const unsigned t = threadIdx.x + seed;
  unsigned b = t * 0x9e3779b9u + 1;
  u64 B = ((u64)b << 32) | (t + 7);
  u64 a0 = t, a1 = t + 1, a2 = t + 2, a3 = t + 3, a4 = t + 4, a5 = t + 5, a6 = t + 6, a7 = t + 7;
  unsigned c0 = t, c1 = t + 1, c2 = t + 2, c3 = t + 3, c4 = t + 4, c5 = t + 5, c6 = t + 6, c7 = t + 7;
  __syncthreads();
  const u64 s = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < ITERS; ++i) {
    if constexpr (OP == 0) {  // v_add_u32
#define a0 c0
#define a1 c1
#define a2 c2
#define a3 c3
#define a4 c4
#define a5 c5
#define a6 c6
#define a7 c7
      CHAIN8("v_add_u32 %0, %0, %1")
    } else if constexpr (OP == 1) {
      CHAIN8("v_xor_b32 %0, %0, %1")
    } else if constexpr (OP == 2) {
      CHAIN8("v_mul_lo_u32 %0, %0, %1")
    } else if constexpr (OP == 3) {
      CHAIN8("v_mul_hi_u32 %0, %0, %1")
    } else if constexpr (OP == 4) {
      CHAIN8("v_alignbyte_b32 %0, %0, %1, %1")
    } else if constexpr (OP == 5) {
      CHAIN8("v_alignbit_b32 %0, %0, %1, 13")
    } else if constexpr (OP == 6) {
      CHAIN8("v_add3_u32 %0, %0, %1, %1")
#undef a0
#undef a1
#undef a2
#undef a3
#undef a4
#undef a5
#undef a6
#undef a7
    } else if constexpr (OP == 7) {  // 64-bit add (gfx940+)
      asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(a0) : "v"(B));
      asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(a1) : "v"(B));
      asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(a2) : "v"(B));
      asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(a3) : "v"(B));
      asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(a4) : "v"(B));
      asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(a5) : "v"(B));
      asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(a6) : "v"(B));
      asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(a7) : "v"(B));
    } else if constexpr (OP == 8) {  // 32x32 -> 64 multiply-add
      asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %1, %0" : "+v"(a0) : "v"(b) : "s0", "s1");
      asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %1, %0" : "+v"(a1) : "v"(b) : "s0", "s1");
      asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %1, %0" : "+v"(a2) : "v"(b) : "s0", "s1");
      asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %1, %0" : "+v"(a3) : "v"(b) : "s0", "s1");
      asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %1, %0" : "+v"(a4) : "v"(b) : "s0", "s1");
      asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %1, %0" : "+v"(a5) : "v"(b) : "s0", "s1");
      asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %1, %0" : "+v"(a6) : "v"(b) : "s0", "s1");
      asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %1, %0" : "+v"(a7) : "v"(b) : "s0", "s1");
    } else if constexpr (OP == 9) {  // 64-bit shift
      asm volatile("v_lshrrev_b64 %0, 7, %0" : "+v"(a0));
      asm volatile("v_lshrrev_b64 %0, 7, %0" : "+v"(a1));
      asm volatile("v_lshrrev_b64 %0, 7, %0" : "+v"(a2));
      asm volatile("v_lshrrev_b64 %0, 7, %0" : "+v"(a3));
      asm volatile("v_lshrrev_b64 %0, 7, %0" : "+v"(a4));
      asm volatile("v_lshrrev_b64 %0, 7, %0" : "+v"(a5));
      asm volatile("v_lshrrev_b64 %0, 7, %0" : "+v"(a6));
      asm volatile("v_lshrrev_b64 %0, 7, %0" : "+v"(a7));
    } else if constexpr (OP == 11) {
#define a0 c0
#define a1 c1
#define a2 c2
#define a3 c3
#define a4 c4
#define a5 c5
#define a6 c6
#define a7 c7
      CHAIN8("v_perm_b32 %0, %0, %1, %1")
    } else if constexpr (OP == 12) {
      CHAIN8("v_bfe_u32 %0, %0, %1, 6")
    } else if constexpr (OP == 13) {
      CHAIN8("v_lshl_add_u32 %0, %0, 2, %1")
#undef a0
#undef a1
#undef a2
#undef a3
#undef a4
#undef a5
#undef a6
#undef a7
    } else if constexpr (OP == 10) {  // the pk 32-bit mul on gfx950, if any: v_mul_u32_u24
      asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(c0) : "v"(b));
      asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(c1) : "v"(b));
      asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(c2) : "v"(b));
      asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(c3) : "v"(b));
      asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(c4) : "v"(b));
      asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(c5) : "v"(b));
      asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(c6) : "v"(b));
      asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(c7) : "v"(b));
    }
  }
  const u64 e = __builtin_amdgcn_s_memtime();
  const unsigned w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if ((threadIdx.x & 63) == 0) cyc[w] = e - s;
  const u64 acc = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ c0 ^ c1 ^ c2 ^ c3 ^ c4 ^ c5 ^ c6 ^ c7;
  if (acc == 0x1234567) sink[0] = 1;  // keeps the chains alive
}

static const char *kNames[] = {"v_add_u32",    "v_xor_b32",       "v_mul_lo_u32",   "v_mul_hi_u32",
                               "v_alignbyte_b32", "v_alignbit_b32", "v_add3_u32",     "v_lshl_add_u64",
                               "v_mad_u64_u32", "v_lshrrev_b64",   "v_mul_u32_u24",  "v_perm_b32",
                               "v_bfe_u32",     "v_lshl_add_u32"};

template <int OP>
static void run(int cus, int w_per_simd, unsigned long long *d_cyc, unsigned *d_sink) {
  const int threads = 64 * 4 * w_per_simd;  // one workgroup per CU: W waves on each SIMD
  const int nw = cus * 4 * w_per_simd;
  k_probe<OP><<<cus, threads>>>(d_cyc, d_sink, 1);  // warm-up
  hipDeviceSynchronize();
  k_probe<OP><<<cus, threads>>>(d_cyc, d_sink, 2);
  hipDeviceSynchronize();
  std::vector<unsigned long long> c(nw);
  hipMemcpy(c.data(), d_cyc, nw * 8, hipMemcpyDeviceToHost);
  double sum = 0;
  for (auto v : c) sum += (double)v;
  const double wave_cycles = sum / nw;
  const double insts = 8.0 * ITERS;
  // s_memtime counts the shader clock: cycles per instruction per SIMD
  printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"cycles_per_inst_per_simd\": %.3f, "
         "\"cycles_per_inst_one_wave\": %.3f}\n",
         kNames[OP], w_per_simd, wave_cycles / (insts * w_per_simd), wave_cycles / insts);
}

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  unsigned long long *d_cyc;
  unsigned *d_sink;
  hipMalloc(&d_cyc, (size_t)cus * 4 * 16 * 8);
  hipMalloc(&d_sink, 4);
  for (int w : {1, 2, 4}) {
    run<0>(cus, w, d_cyc, d_sink);
    run<1>(cus, w, d_cyc, d_sink);
    run<2>(cus, w, d_cyc, d_sink);
    run<3>(cus, w, d_cyc, d_sink);
    run<4>(cus, w, d_cyc, d_sink);
    run<5>(cus, w, d_cyc, d_sink);
    run<6>(cus, w, d_cyc, d_sink);
    run<7>(cus, w, d_cyc, d_sink);
    run<8>(cus, w, d_cyc, d_sink);
    run<9>(cus, w, d_cyc, d_sink);
    run<10>(cus, w, d_cyc, d_sink);
    run<11>(cus, w, d_cyc, d_sink);
    run<12>(cus, w, d_cyc, d_sink);
    run<13>(cus, w, d_cyc, d_sink);
  }
  return 0;
}
