// valu_rate.hip -- measurement helper (not product code): the SIMD's fp32
// VALU issue rate on gfx950, to price `valu_issue_frac` (bench.py) in cycles
// per wave64 instruction.  Each wave runs CH independent v_fma_f32 chains
// (or v_pk_fma_f32 with PK) for ITERS x 16 steps; the grid puts W waves on
// each of the 1 024 SIMDs (256 CUs x 4).  Reported per configuration:
// SIMD cycles per wave64 instruction = kernel time x clock / (instructions
// per SIMD), the clock measured inside the kernel (s_memtime over
// s_memrealtime, 100 MHz).  Also one dependent chain (CH = 1, W = 1): the
// dependent-issue latency.
//   make -C tools/hip valu_rate && tools/hip/valu_rate > out.json
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                        \
    }                                                                      \
  } while (0)

typedef float f2 __attribute__((ext_vector_type(2)));

template <int CH, bool PK>
__global__ __launch_bounds__(256) void valu_kernel(float* out, unsigned long long* clk, int iters, float s) {
  unsigned long long t0 = 0, r0 = 0;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    t0 = __builtin_amdgcn_s_memtime();
    r0 = __builtin_amdgcn_s_memrealtime();
  }
  if constexpr (PK) {
    f2 a[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) a[c] = f2{(float)threadIdx.x * 1e-7f + c, (float)c * 0.5f};
    const f2 m = f2{s, s * 0.5f}, k = f2{1e-7f, 2e-7f};
    for (int i = 0; i < iters; ++i) {
#pragma unroll
      for (int u = 0; u < 16; ++u)
#pragma unroll
        for (int c = 0; c < CH; ++c) {
          a[c] = __builtin_elementwise_fma(a[c], m, k);
          asm volatile("" : "+v"(a[c]));
        }
    }
    float r = 0.f;
#pragma unroll
    for (int c = 0; c < CH; ++c) r += a[c].x + a[c].y;
    if (r == 12345.678f) out[threadIdx.x] = r;
  } else {
    float a[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) a[c] = (float)threadIdx.x * 1e-7f + c;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
      for (int u = 0; u < 16; ++u)
#pragma unroll
        for (int c = 0; c < CH; ++c) {
          a[c] = __builtin_fmaf(a[c], s, 1e-7f);
          asm volatile("" : "+v"(a[c]));
        }
    }
    float r = 0.f;
#pragma unroll
    for (int c = 0; c < CH; ++c) r += a[c];
    if (r == 12345.678f) out[threadIdx.x] = r;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    clk[0] = __builtin_amdgcn_s_memtime() - t0;
    clk[1] = __builtin_amdgcn_s_memrealtime() - r0;
  }
}

// one instruction (inline asm, operand 0 = the chain register, 1 = a second
// VGPR, 2 = an SGPR) on 8 independent chains per step
#define OPK(NAME, ASM)                                                                 \
  __global__ __launch_bounds__(256) void op_##NAME(float* out, unsigned long long* clk, int iters, float s) { \
    float a[8];                                                                        \
    _Pragma("unroll") for (int c = 0; c < 8; ++c) a[c] = (float)threadIdx.x * 1e-7f + c; \
    const float bb = s * 0.5f;                                                         \
    for (int i = 0; i < iters; ++i) {                                                  \
      _Pragma("unroll") for (int u = 0; u < 16; ++u)                                   \
      _Pragma("unroll") for (int c = 0; c < 8; ++c) asm volatile(ASM : "+v"(a[c]) : "v"(bb), "s"(s) : "vcc"); \
    }                                                                                  \
    float r = 0.f;                                                                     \
    _Pragma("unroll") for (int c = 0; c < 8; ++c) r += a[c];                           \
    if (r == 12345.678f) out[threadIdx.x] = r;                                         \
  }
OPK(v_mul_f32, "v_mul_f32 %0, %0, %1")
OPK(v_add_u32, "v_add_u32 %0, %0, %1")
OPK(v_and_b32, "v_and_b32 %0, %0, %1")
OPK(v_min_f32, "v_min_f32 %0, %0, %1")
OPK(v_mov_b32, "v_mov_b32 %0, %1")
OPK(v_rndne_f32, "v_rndne_f32 %0, %0")
OPK(v_cvt_i32_f32, "v_cvt_i32_f32 %0, %0")
OPK(v_ldexp_f32, "v_ldexp_f32 %0, %0, %1")
OPK(v_ffbl_b32, "v_ffbl_b32 %0, %0")
OPK(v_cmp_lt_f32, "v_cmp_lt_f32 vcc, %0, %1")
OPK(v_exp_f32, "v_exp_f32 %0, %0")
OPK(v_sub_f32, "v_sub_f32 %0, %0, %1")
OPK(v_lshlrev_b32, "v_lshlrev_b32 %0, 3, %0")
OPK(v_or_b32, "v_or_b32 %0, %0, %1")
OPK(v_bfe_u32, "v_bfe_u32 %0, %0, 3, 9")
OPK(v_max_f32, "v_max_f32 %0, %0, %1")
OPK(v_mul_lo_u32, "v_mul_lo_u32 %0, %0, %1")
OPK(v_cvt_f32_u32, "v_cvt_f32_u32 %0, %0")
OPK(v_sqrt_f32, "v_sqrt_f32 %0, %0")
OPK(v_rcp_f32, "v_rcp_f32 %0, %0")
OPK(v_mad_u32_u24, "v_mad_u32_u24 %0, %0, %1, %0")
OPK(v_fmac_f32, "v_fmac_f32 %0, %1, %1")
OPK(v_min_u32, "v_min_u32 %0, %0, %1")
OPK(v_lshl_add_u32, "v_lshl_add_u32 %0, %0, 4, %1")
__global__ __launch_bounds__(256) void op_v_cndmask_b32(float* out, unsigned long long* clk, int iters, float s) {
  float a[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) a[c] = (float)threadIdx.x * 1e-7f + c;
  const float bb = s * 0.5f;
  const unsigned long long mask = (unsigned long long)iters * 0x9E3779B97F4A7C15ull;  // a loop-invariant SGPR pair
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int u = 0; u < 16; ++u)
#pragma unroll
      for (int c = 0; c < 8; ++c) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(a[c]) : "v"(bb), "s"(mask));
  }
  float r = 0.f;
#pragma unroll
  for (int c = 0; c < 8; ++c) r += a[c];
  if (r == 12345.678f) out[threadIdx.x] = r;
}

// packed / 64-bit operations on a register pair per chain
#define OPK2(NAME, ASM)                                                                \
  __global__ __launch_bounds__(256) void op_##NAME(float* out, unsigned long long* clk, int iters, float s) { \
    f2 a[8];                                                                           \
    _Pragma("unroll") for (int c = 0; c < 8; ++c) a[c] = f2{(float)threadIdx.x * 1e-7f + c, 0.5f * c}; \
    const f2 bb = f2{s * 0.5f, s * 0.25f};                                             \
    for (int i = 0; i < iters; ++i) {                                                  \
      _Pragma("unroll") for (int u = 0; u < 16; ++u)                                   \
      _Pragma("unroll") for (int c = 0; c < 8; ++c) asm volatile(ASM : "+v"(a[c]) : "v"(bb)); \
    }                                                                                  \
    float r = 0.f;                                                                     \
    _Pragma("unroll") for (int c = 0; c < 8; ++c) r += a[c].x + a[c].y;                \
    if (r == 12345.678f) out[threadIdx.x] = r;                                         \
  }
OPK2(v_pk_mul_f32, "v_pk_mul_f32 %0, %0, %1")
OPK2(v_pk_add_f32, "v_pk_add_f32 %0, %0, %1")
OPK2(v_lshl_add_u64, "v_lshl_add_u64 %0, %0, 0, %1")
OPK2(v_cmp_eq_u64, "v_cmp_eq_u64 s[0:1], %0, %1")

// Compiler-emitted forms (no inline-asm instruction, so no per-instruction
// s_nop pad after it: the asm OPK kernels above get an `s_nop 0` after every
// instruction, these one per 8-chain step, the same for every op): the four
// plain ops of the blend's record step, and fma / mul (add) alternating, at 8 waves per
// SIMD.  Round 6: settles whether a v_fma_f32 costs twice a v_mul_f32.
#define BIK(NAME, EXPR)                                                                \
  __global__ __launch_bounds__(256) void bi_##NAME(float* out, unsigned long long* clk, int iters, float s) { \
    float a[8];                                                                        \
    _Pragma("unroll") for (int c = 0; c < 8; ++c) a[c] = (float)threadIdx.x * 1e-7f + c; \
    const float k = s * 1e-7f;                                                         \
    for (int i = 0; i < iters; ++i) {                                                  \
      _Pragma("unroll") for (int u = 0; u < 16; ++u)                                   \
      _Pragma("unroll") for (int c = 0; c < 8; ++c) {                                  \
        const float x = a[c];                                                          \
        a[c] = (EXPR);                                                                 \
        asm volatile("" : "+v"(a[c]));                                                 \
      }                                                                                \
    }                                                                                  \
    float r = 0.f;                                                                     \
    _Pragma("unroll") for (int c = 0; c < 8; ++c) r += a[c];                           \
    if (r == 12345.678f) out[threadIdx.x] = r;                                         \
  }
BIK(fma, __builtin_fmaf(x, s, k))
BIK(mul, x * s)
BIK(add, x + s)
BIK(fma_mul, ((c & 1) ? x * s : __builtin_fmaf(x, s, k)))
BIK(fma_add, ((c & 1) ? x + s : __builtin_fmaf(x, s, k)))
// the operand kinds (round 6): a per-lane (VGPR) multiplier, an inline
// constant, a literal; fma with every source a VGPR
#define BIV(NAME, EXPR)                                                                \
  __global__ __launch_bounds__(256) void bv_##NAME(float* out, unsigned long long* clk, int iters, float s) { \
    float a[8];                                                                        \
    _Pragma("unroll") for (int c = 0; c < 8; ++c) a[c] = (float)threadIdx.x * 1e-7f + c; \
    float v = s * (1.0f + (float)threadIdx.x * 1e-9f), w = v * 1e-7f;                   \
    asm volatile("" : "+v"(v), "+v"(w));                                               \
    for (int i = 0; i < iters; ++i) {                                                  \
      _Pragma("unroll") for (int u = 0; u < 16; ++u)                                   \
      _Pragma("unroll") for (int c = 0; c < 8; ++c) {                                  \
        const float x = a[c];                                                          \
        a[c] = (EXPR);                                                                 \
        asm volatile("" : "+v"(a[c]));                                                 \
      }                                                                                \
    }                                                                                  \
    float r = 0.f;                                                                     \
    _Pragma("unroll") for (int c = 0; c < 8; ++c) r += a[c];                           \
    if (r == 12345.678f) out[threadIdx.x] = r;                                         \
  }
BIV(mul_vgpr, x * v)
BIV(add_vgpr, x + v)
BIV(mul_inline, x * 0.5f)
BIV(mul_literal, x * 0.99987f)
BIV(fma_vgpr, __builtin_fmaf(x, v, w))
BIV(min_vgpr, __builtin_fminf(x, v))

template <int CH, bool PK>
static void run(const char* name, int waves_per_simd, int iters, float* out, unsigned long long* clk, bool first) {
  const int blocks = 256 * waves_per_simd;  // 4 waves per block: one per SIMD
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int w = 0; w < 3; ++w) valu_kernel<CH, PK><<<blocks, 256>>>(out, clk, iters, 0.999f);
  CK(hipDeviceSynchronize());
  const int reps = 10;
  CK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r) valu_kernel<CH, PK><<<blocks, 256>>>(out, clk, iters, 0.999f);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, e0, e1));
  unsigned long long h[2];
  CK(hipMemcpy(h, clk, sizeof(h), hipMemcpyDeviceToHost));
  const double ghz = h[1] ? (double)h[0] / (double)h[1] * 0.1 : 0.0;  // shader ticks per 10 ns
  const double t = ms * 1e-3 / reps;
  // wave64 instructions per SIMD (each of the 1 024 SIMDs runs waves_per_simd waves)
  const double insts = (double)waves_per_simd * iters * 16 * CH;
  const double cyc = t * ghz * 1e9 / insts;
  std::printf("%s{\"op\": \"%s\", \"chains\": %d, \"waves_per_simd\": %d, \"us\": %.2f, \"clock_ghz\": %.3f, "
              "\"simd_cycles_per_inst\": %.3f}",
              first ? "" : ",\n", name, CH, waves_per_simd, t * 1e6, ghz, cyc);
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
}

static void run_op(const char* name, void (*k)(float*, unsigned long long*, int, float), float* out,
                   unsigned long long* clk) {
  const int w = 8, iters = 1024, blocks = 256 * w;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int r = 0; r < 2; ++r) hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, clk, iters, 0.999f);
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0));
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, clk, iters, 0.999f);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double t = ms * 1e-3 / 5, insts = (double)w * iters * 16 * 8;
  std::printf(",\n{\"op\": \"%s\", \"chains\": 8, \"waves_per_simd\": %d, \"us\": %.2f, "
              "\"simd_cycles_per_inst_at_2.4GHz\": %.3f}", name, w, t * 1e6, t * 2.4e9 / insts);
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
}

int main() {
  float* out;
  unsigned long long* clk;
  CK(hipMalloc(&out, 4096));
  CK(hipMalloc(&clk, 16));
  const int iters = 2048;
  std::printf("[\n");
  bool first = true;
  for (int w : {1, 2, 4, 8}) {
    run<8, false>("v_fma_f32", w, iters, out, clk, first);
    first = false;
  }
  for (int w : {1, 2, 4, 8}) run<2, false>("v_fma_f32", w, iters, out, clk, false);
  run<1, false>("v_fma_f32", 1, iters, out, clk, false);
  for (int w : {1, 4, 8}) run<8, true>("v_pk_fma_f32", w, iters, out, clk, false);
#define RUN_OP(N) run_op(#N, op_##N, out, clk)
  RUN_OP(v_mul_f32);
  RUN_OP(v_add_u32);
  RUN_OP(v_and_b32);
  RUN_OP(v_min_f32);
  RUN_OP(v_mov_b32);
  RUN_OP(v_rndne_f32);
  RUN_OP(v_cvt_i32_f32);
  RUN_OP(v_ldexp_f32);
  RUN_OP(v_ffbl_b32);
  RUN_OP(v_cmp_lt_f32);
  RUN_OP(v_exp_f32);
  RUN_OP(v_sub_f32);
  RUN_OP(v_lshlrev_b32);
  RUN_OP(v_or_b32);
  RUN_OP(v_bfe_u32);
  RUN_OP(v_max_f32);
  RUN_OP(v_mul_lo_u32);
  RUN_OP(v_cvt_f32_u32);
  RUN_OP(v_sqrt_f32);
  RUN_OP(v_rcp_f32);
  RUN_OP(v_mad_u32_u24);
  RUN_OP(v_fmac_f32);
  RUN_OP(v_min_u32);
  RUN_OP(v_lshl_add_u32);
  RUN_OP(v_cndmask_b32);
  RUN_OP(v_pk_mul_f32);
  RUN_OP(v_pk_add_f32);
  RUN_OP(v_lshl_add_u64);
  RUN_OP(v_cmp_eq_u64);
  run_op("bi_v_fma_f32", bi_fma, out, clk);
  run_op("bi_v_mul_f32", bi_mul, out, clk);
  run_op("bi_v_add_f32", bi_add, out, clk);
  run_op("bi_fma_mul_alternating", bi_fma_mul, out, clk);
  run_op("bi_fma_add_alternating", bi_fma_add, out, clk);
  run_op("bv_v_mul_f32_vgpr", bv_mul_vgpr, out, clk);
  run_op("bv_v_add_f32_vgpr", bv_add_vgpr, out, clk);
  run_op("bv_v_mul_f32_inline", bv_mul_inline, out, clk);
  run_op("bv_v_mul_f32_literal", bv_mul_literal, out, clk);
  run_op("bv_v_fma_f32_vgpr", bv_fma_vgpr, out, clk);
  run_op("bv_v_min_f32_vgpr", bv_min_vgpr, out, clk);
  std::printf("\n]\n");
  return 0;
}
