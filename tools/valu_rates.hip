// VALU issue-rate microbenchmark, second set (diagnostic tool, not product code): the
// instruction forms the trace kernel's hash / division / sqrt sequences are built from.
// 8 independent chains per lane, 8 waves per SIMD (2048 x 256 threads on 256 CUs); cycles
// per wave64 instruction per SIMD from the s_memtime / s_memrealtime clock of block 0.
//   hipcc --offload-arch=gfx950 -O3 tools/valu_rates.hip -o tools/valu_rates && ./tools/valu_rates
#include <hip/hip_runtime.h>
#include <cstdio>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int ITERS = 2048;
typedef float f2 __attribute__((ext_vector_type(2)));

__device__ inline float tof(float v) { return v; }
__device__ inline float tof(unsigned v) { return (float)v; }
__device__ inline float tof(unsigned long long v) { return (float)v; }
__device__ inline float tof(f2 v) { return v.x + v.y; }
__device__ inline float tof(double v) { return (float)v; }

#define REP8(S, A) S(A##0) S(A##1) S(A##2) S(A##3) S(A##4) S(A##5) S(A##6) S(A##7)

// T: register type of the chains, INIT(i): initial value, ASM: one instruction on "%0"
#define KER(NAME, T, INIT, ASM)                                                               \
    __global__ __launch_bounds__(256) void NAME(float* out, unsigned long long* clk) {         \
        T a0 = INIT(0), a1 = INIT(1), a2 = INIT(2), a3 = INIT(3), a4 = INIT(4), a5 = INIT(5),   \
          a6 = INIT(6), a7 = INIT(7);                                                         \
        const float x = threadIdx.x * 0.5f + 1.0f, y = threadIdx.x * 0.25f + 1.0f;              \
        const unsigned ux = threadIdx.x * 7u + 3u;                                            \
        const f2 px = {x, y};                                                                 \
        const unsigned long long m64 = __builtin_amdgcn_read_exec() ^ 0x5555555555555555ull; \
        const float sf = __builtin_amdgcn_readfirstlane(threadIdx.x) * 0.5f; unsigned long long mm = 0; (void)mm; (void)m64; (void)sf; \
        unsigned long long t0 = 0, r0 = 0;                                                    \
        if (blockIdx.x == 0 && threadIdx.x == 0) {                                            \
            t0 = __builtin_amdgcn_s_memtime();                                                \
            r0 = __builtin_amdgcn_s_memrealtime();                                            \
        }                                                                                     \
        for (int i = 0; i < ITERS; ++i) {                                                     \
            _Pragma("unroll") for (int k = 0; k < 1; ++k) {                                  \
                REP8(STEP_##NAME, a)                                                          \
            }                                                                                 \
        }                                                                                     \
        if (blockIdx.x == 0 && threadIdx.x == 0) {                                            \
            clk[0] = __builtin_amdgcn_s_memtime() - t0;                                       \
            clk[1] = __builtin_amdgcn_s_memrealtime() - r0;                                   \
        }                                                                                     \
        out[blockIdx.x * 256 + threadIdx.x] = tof(a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7);     \
    }

#define FI(i) (threadIdx.x * 0.5f + (float)(i))
#define UI(i) (threadIdx.x * 3u + (unsigned)(i))
#define PI(i) (f2{threadIdx.x * 0.5f + (float)(i), 1.0f})
#define LI(i) ((unsigned long long)threadIdx.x * 3ull + (unsigned long long)(i))
typedef float f1;
typedef unsigned u1;
typedef unsigned long long l1;
#define F1(i) FI(i)
#define U1(i) UI(i)
#define L1(i) LI(i)

#define STEP_k_fma(a) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(a) : "v"(x), "v"(y));
KER(k_fma, f1, F1, _)
#define STEP_k_mul_lo(a) asm volatile("v_mul_lo_u32 %0, %1, %0" : "+v"(a) : "v"(ux));
KER(k_mul_lo, u1, U1, _)
#define STEP_k_mul_hi(a) asm volatile("v_mul_hi_u32 %0, %1, %0" : "+v"(a) : "v"(ux));
KER(k_mul_hi, u1, U1, _)
#define STEP_k_mul_u24(a) asm volatile("v_mul_u32_u24 %0, %1, %0" : "+v"(a) : "v"(ux));
KER(k_mul_u24, u1, U1, _)
#define STEP_k_mad_u24(a) asm volatile("v_mad_u32_u24 %0, %1, %0, %1" : "+v"(a) : "v"(ux));
KER(k_mad_u24, u1, U1, _)
#define STEP_k_mad_u64(a) asm volatile("v_mad_u64_u32 %0, vcc, %1, %1, %0" : "+v"(a) : "v"(ux) : "vcc");
KER(k_mad_u64, l1, L1, _)
#define STEP_k_lshl_add(a) asm volatile("v_lshl_add_u32 %0, %0, 24, %1" : "+v"(a) : "v"(ux));
KER(k_lshl_add, u1, U1, _)
#define STEP_k_xor(a) asm volatile("v_xor_b32 %0, %1, %0" : "+v"(a) : "v"(ux));
KER(k_xor, u1, U1, _)
#define STEP_k_xor_sdwa(a) asm volatile("v_xor_b32_sdwa %0, %0, %0 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1" : "+v"(a));
KER(k_xor_sdwa, u1, U1, _)
#define STEP_k_pk_fma(a) asm volatile("v_pk_fma_f32 %0, %1, %1, %0" : "+v"(a) : "v"(px));
KER(k_pk_fma, f2, PI, _)
#define STEP_k_pk_mul(a) asm volatile("v_pk_mul_f32 %0, %1, %0" : "+v"(a) : "v"(px));
KER(k_pk_mul, f2, PI, _)
#define STEP_k_pk_add(a) asm volatile("v_pk_add_f32 %0, %1, %0" : "+v"(a) : "v"(px));
KER(k_pk_add, f2, PI, _)
#define STEP_k_rcp(a) asm volatile("v_rcp_f32 %0, %0" : "+v"(a));
KER(k_rcp, f1, F1, _)
#define STEP_k_sqrt(a) asm volatile("v_sqrt_f32 %0, %0" : "+v"(a));
KER(k_sqrt, f1, F1, _)
#define STEP_k_rsq(a) asm volatile("v_rsq_f32 %0, %0" : "+v"(a));
KER(k_rsq, f1, F1, _)
#define STEP_k_sin(a) asm volatile("v_sin_f32 %0, %0" : "+v"(a));
KER(k_sin, f1, F1, _)
#define STEP_k_div_scale(a) asm volatile("v_div_scale_f32 %0, vcc, %1, %2, %0" : "+v"(a) : "v"(x), "v"(y) : "vcc");
KER(k_div_scale, f1, F1, _)
#define STEP_k_div_fmas(a) asm volatile("v_div_fmas_f32 %0, %1, %2, %0" : "+v"(a) : "v"(x), "v"(y));
KER(k_div_fmas, f1, F1, _)
#define STEP_k_div_fixup(a) asm volatile("v_div_fixup_f32 %0, %0, %1, %2" : "+v"(a) : "v"(x), "v"(y));
KER(k_div_fixup, f1, F1, _)
#define STEP_k_cvt_f32_u32(a) asm volatile("v_cvt_f32_u32 %0, %0" : "+v"(a));
KER(k_cvt_f32_u32, f1, F1, _)
#define STEP_k_cndmask(a) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a) : "v"(x));
KER(k_cndmask, f1, F1, _)
#define STEP_k_ldexp(a) asm volatile("v_ldexp_f32 %0, %0, 3" : "+v"(a));
KER(k_ldexp, f1, F1, _)
#define STEP_k_frexp_exp(a) asm volatile("v_frexp_exp_i32_f32 %0, %0" : "+v"(a));
KER(k_frexp_exp, f1, F1, _)
#define STEP_k_med3(a) asm volatile("v_med3_f32 %0, %0, %1, %2" : "+v"(a) : "v"(x), "v"(y));
KER(k_med3, f1, F1, _)
#define STEP_k_perm(a) asm volatile("v_perm_b32 %0, %0, %1, %1" : "+v"(a) : "v"(ux));
KER(k_perm, u1, U1, _)
#define STEP_k_alignbit(a) asm volatile("v_alignbit_b32 %0, %0, %1, 16" : "+v"(a) : "v"(ux));
KER(k_alignbit, u1, U1, _)

#define STEP_k_cnd_sgpr(a) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(a) : "v"(x), "s"(m64));
#define KERM(NAME) KER(NAME, f1, F1, _)
#define STEP_k_add_u32(a) asm volatile("v_add_u32 %0, %1, %0" : "+v"(a) : "v"(ux));
KER(k_add_u32, u1, U1, _)
#define STEP_k_lshr(a) asm volatile("v_lshrrev_b32 %0, 16, %0" : "+v"(a));
KER(k_lshr, u1, U1, _)
#define STEP_k_and(a) asm volatile("v_and_b32 %0, %1, %0" : "+v"(a) : "v"(ux));
KER(k_and, u1, U1, _)
#define STEP_k_mov(a) asm volatile("v_mov_b32 %0, %1" : "=v"(a) : "v"(ux));
KER(k_mov, u1, U1, _)
#define STEP_k_mul_f32(a) asm volatile("v_mul_f32 %0, %1, %0" : "+v"(a) : "v"(x));
KER(k_mul_f32, f1, F1, _)
#define STEP_k_sub_f32(a) asm volatile("v_sub_f32 %0, %1, %0" : "+v"(a) : "v"(x));
KER(k_sub_f32, f1, F1, _)
#define STEP_k_max_f32(a) asm volatile("v_max_f32 %0, %1, %0" : "+v"(a) : "v"(x));
KER(k_max_f32, f1, F1, _)
#define STEP_k_fma_abs(a) asm volatile("v_fma_f32 %0, |%1|, %2, -%0" : "+v"(a) : "v"(x), "v"(y));
KER(k_fma_abs, f1, F1, _)
#define STEP_k_fma_sgpr(a) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(a) : "v"(x), "s"(sf));
KER(k_fma_sgpr, f1, F1, _)
#define STEP_k_fma_lit(a) asm volatile("v_fmaak_f32 %0, %1, %0, 0x3f8ccccd" : "+v"(a) : "v"(x));
KER(k_fma_lit, f1, F1, _)
#define STEP_k_cmp_lt(a) asm volatile("v_cmp_lt_f32_e64 %0, %1, %2" : "=s"(mm) : "v"(a), "v"(x)); a += 0;
#define STEP_k_bfi(a) asm volatile("v_bfi_b32 %0, %1, %0, %1" : "+v"(a) : "v"(ux));
KER(k_bfi, u1, U1, _)
#define STEP_k_cmp_class(a) asm volatile("v_cmp_class_f32_e64 %0, %1, %2" : "=s"(mm) : "v"(a), "v"(ux)); a += 0;
#define STEP_k_min3(a) asm volatile("v_min3_f32 %0, %0, %1, %2" : "+v"(a) : "v"(x), "v"(y));
KER(k_min3, f1, F1, _)
#define STEP_k_rndne(a) asm volatile("v_rndne_f32 %0, %0" : "+v"(a));
KER(k_rndne, f1, F1, _)
#define STEP_k_cvt_i32(a) asm volatile("v_cvt_i32_f32 %0, %0" : "+v"(a));
KER(k_cvt_i32, f1, F1, _)
KER(k_cnd_sgpr, f1, F1, _)
KER(k_cmp_lt, f1, F1, _)
KER(k_cmp_class, f1, F1, _)

// round 3: the remaining forms of rt_single_kernel's hot path (tools/valu_weighted.py)
typedef double d1;
#define D1(i) ((double)threadIdx.x * 0.5 + (double)(i))
const double dx = 1.5;
#define STEP_k_mul_f64(a) asm volatile("v_mul_f64 %0, %1, %0" : "+v"(a) : "v"(dx));
KER(k_mul_f64, d1, D1, _)
#define STEP_k_fma_f64(a) asm volatile("v_fma_f64 %0, %1, %1, %0" : "+v"(a) : "v"(dx));
KER(k_fma_f64, d1, D1, _)
#define STEP_k_cvt_f64_f32(a) { double t_; asm volatile("v_cvt_f64_f32 %0, %1" : "=v"(t_) : "v"(a)); asm volatile("" :: "v"(t_)); }
KER(k_cvt_f64_f32, f1, F1, _)
#define STEP_k_cvt_f32_f64(a) { float t_; asm volatile("v_cvt_f32_f64 %0, %1" : "=v"(t_) : "v"(a)); asm volatile("" :: "v"(t_)); }
KER(k_cvt_f32_f64, d1, D1, _)
#define STEP_k_cvt_u32_f32(a) asm volatile("v_cvt_u32_f32 %0, %0" : "+v"(a));
KER(k_cvt_u32_f32, f1, F1, _)
#define STEP_k_fmac(a) asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(a) : "v"(x), "v"(y));
KER(k_fmac, f1, F1, _)
#define STEP_k_fmamk(a) asm volatile("v_fmamk_f32 %0, %0, 0x3f8ccccd, %1" : "+v"(a) : "v"(x));
KER(k_fmamk, f1, F1, _)
#define STEP_k_add_f32(a) asm volatile("v_add_f32 %0, %1, %0" : "+v"(a) : "v"(x));
KER(k_add_f32, f1, F1, _)
#define STEP_k_bitop3(a) asm volatile("v_bitop3_b32 %0, %0, %1, %1 bitop3:0x96" : "+v"(a) : "v"(ux));
KER(k_bitop3, u1, U1, _)
#define STEP_k_lshl_or(a) asm volatile("v_lshl_or_b32 %0, %0, 3, %1" : "+v"(a) : "v"(ux));
KER(k_lshl_or, u1, U1, _)
#define STEP_k_min3_u32(a) asm volatile("v_min3_u32 %0, %0, %1, %1" : "+v"(a) : "v"(ux));
KER(k_min3_u32, u1, U1, _)
#define STEP_k_max_i32(a) asm volatile("v_max_i32 %0, %1, %0" : "+v"(a) : "v"(ux));
KER(k_max_i32, u1, U1, _)
#define STEP_k_bfe(a) asm volatile("v_bfe_u32 %0, %0, 3, 7" : "+v"(a));
KER(k_bfe, u1, U1, _)
#define STEP_k_lshl_add_u64(a) asm volatile("v_lshl_add_u64 %0, %0, 4, %0" : "+v"(a));
KER(k_lshl_add_u64, l1, L1, _)
#define STEP_k_mov_b64(a) asm volatile("v_mov_b64 %0, %1" : "=v"(a) : "v"(dx));
KER(k_mov_b64, d1, D1, _)
#define STEP_k_cmp_u32_e32(a) asm volatile("v_cmp_gt_u32_e32 vcc, %0, %1" :: "v"(a), "v"(ux) : "vcc");
KER(k_cmp_u32_e32, u1, U1, _)
#define STEP_k_cmp_f32_e32(a) asm volatile("v_cmp_gt_f32_e32 vcc, %0, %1" :: "v"(a), "v"(x) : "vcc");
KER(k_cmp_f32_e32, f1, F1, _)
#define STEP_k_cnd_vcc(a) asm volatile("s_mov_b64 vcc, %1\n\tv_cndmask_b32_e32 %0, %0, %2, vcc" : "+v"(a) : "s"(m64), "v"(x) : "vcc");
KER(k_cnd_vcc, f1, F1, _)
#define STEP_k_readfirstlane(a) { unsigned t_; asm volatile("v_readfirstlane_b32 %0, %1" : "=s"(t_) : "v"(a)); asm volatile("" :: "s"(t_)); }
KER(k_readfirstlane, u1, U1, _)
#define STEP_k_mul_lo_mix(a) asm volatile("v_mul_lo_u32 %0, %1, %0\n\tv_add_u32 %0, %1, %0" : "+v"(a) : "v"(ux));
KER(k_mul_lo_mix, u1, U1, _)

template <typename F>
int run(const char* name, F launch, float* d_out, unsigned long long* d_clk, int blocks) {
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    launch();
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(e0));
    for (int r = 0; r < 5; ++r) launch();
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    ms /= 5;
    unsigned long long clk[2];
    CHECK(hipMemcpy(clk, d_clk, sizeof(clk), hipMemcpyDeviceToHost));
    const double ghz = (double)clk[0] / ((double)clk[1] / 100e6) / 1e9;
    const double instr = blocks * 4.0 * ITERS * 8;          // wave-instructions per launch
    const double simd_cycles = ms * 1e-3 * ghz * 1e9 * 1024;  // 256 CUs x 4 SIMDs
    printf("%-18s %8.3f ms  clk %.2f GHz  %.2f cycles/wave-instr/SIMD\n", name, ms, ghz,
           simd_cycles / instr);
    return 0;
}

#define RUN(K) run(#K, [&] { hipLaunchKernelGGL(K, dim3(blocks), dim3(256), 0, 0, d_out, d_clk); }, d_out, d_clk, blocks)

int main() {
    const int blocks = 2048;
    float* d_out;
    unsigned long long* d_clk;
    CHECK(hipMalloc(&d_out, blocks * 256 * sizeof(float)));
    CHECK(hipMalloc(&d_clk, 16));
    RUN(k_fma); RUN(k_mul_lo); RUN(k_mul_hi); RUN(k_mul_u24); RUN(k_mad_u24); RUN(k_mad_u64);
    RUN(k_lshl_add); RUN(k_xor); RUN(k_xor_sdwa); RUN(k_pk_fma); RUN(k_pk_mul); RUN(k_pk_add);
    RUN(k_rcp); RUN(k_sqrt); RUN(k_rsq); RUN(k_sin); RUN(k_div_scale); RUN(k_div_fmas);
    RUN(k_div_fixup); RUN(k_cvt_f32_u32); RUN(k_cndmask); RUN(k_ldexp); RUN(k_frexp_exp);
    RUN(k_med3); RUN(k_perm); RUN(k_alignbit);
    RUN(k_cnd_sgpr); RUN(k_add_u32); RUN(k_lshr); RUN(k_and); RUN(k_mov); RUN(k_mul_f32); RUN(k_sub_f32);
    RUN(k_max_f32); RUN(k_fma_abs); RUN(k_fma_sgpr); RUN(k_fma_lit); RUN(k_cmp_lt); RUN(k_bfi); RUN(k_cmp_class);
    RUN(k_min3); RUN(k_rndne); RUN(k_cvt_i32);
    RUN(k_mul_f64); RUN(k_fma_f64); RUN(k_cvt_f64_f32); RUN(k_cvt_f32_f64); RUN(k_cvt_u32_f32);
    RUN(k_fmac); RUN(k_fmamk); RUN(k_add_f32); RUN(k_bitop3); RUN(k_lshl_or); RUN(k_min3_u32);
    RUN(k_max_i32); RUN(k_bfe); RUN(k_lshl_add_u64); RUN(k_mov_b64); RUN(k_cmp_u32_e32);
    RUN(k_cmp_f32_e32); RUN(k_cnd_vcc); RUN(k_readfirstlane);
    // (two instructions per step: the pair's cost)
    RUN(k_mul_lo_mix);
    return 0;
}
