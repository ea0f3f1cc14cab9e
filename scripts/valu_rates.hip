// valu_rates.hip — issue cost of the VALU instructions the path tracer's
// kernels are made of, on the card (wave64, 4 waves per SIMD, 8 independent
// chains per wave so latency is hidden).  Prints cycles per wave-instruction
// per SIMD at the measured clock.  A measurement tool, not part of the product.
//
//   hipcc --offload-arch=gfx950 -O3 scripts/valu_rates.hip -o scripts/valu_rates.bin && scripts/valu_rates.bin
#include <hip/hip_runtime.h>
#include <cstdio>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { std::printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)

constexpr int kIters = 4096;

#define BODY8(OP) OP(0) OP(1) OP(2) OP(3) OP(4) OP(5) OP(6) OP(7)

template <int K>
__global__ __launch_bounds__(256) void k_rate(double* out, unsigned seed) {
    double d[8];
    float f[8];
    unsigned u[8];
    unsigned long long w[8];
    for (int i = 0; i < 8; ++i) {
        d[i] = 1.0 + (threadIdx.x + i + seed) * 1e-9;
        f[i] = 1.0f + (threadIdx.x + i + seed) * 1e-6f;
        u[i] = threadIdx.x * 7 + i + seed;
        w[i] = u[i];
    }
    for (int it = 0; it < kIters; ++it) {
#define FMA(i) asm volatile("v_fma_f64 %0, %0, %0, %0" : "+v"(d[i]));
#define MUL(i) asm volatile("v_mul_f64 %0, %0, %0" : "+v"(d[i]));
#define ADD(i) asm volatile("v_add_f64 %0, %0, %0" : "+v"(d[i]));
#define RCP(i) asm volatile("v_rcp_f64 %0, %0" : "+v"(d[i]));
#define RSQ(i) asm volatile("v_rsq_f64 %0, %0" : "+v"(d[i]));
#define DSC(i) asm volatile("v_div_scale_f64 %0, vcc, %0, %0, %0" : "+v"(d[i]) :: "vcc");
#define DFX(i) asm volatile("v_div_fixup_f64 %0, %0, %0, %0" : "+v"(d[i]));
#define MAD64(i) asm volatile("v_mad_u64_u32 %0, s[40:41], %1, %2, 0" : "=v"(w[i]) : "v"(u[i]), "s"(48271u) : "s40", "s41"); u[i] = (unsigned)w[i];
#define MULLO(i) asm volatile("v_mul_lo_u32 %0, %0, %0" : "+v"(u[i]));
#define MULHI(i) asm volatile("v_mul_hi_u32 %0, %0, %0" : "+v"(u[i]));
#define M24(i) asm volatile("v_mul_u32_u24 %0, %0, %0" : "+v"(u[i]));
#define IADD(i) asm volatile("v_add_u32 %0, %0, %0" : "+v"(u[i]));
#define CVT(i) asm volatile("v_cvt_f64_u32 %0, %1" : "=v"(d[i]) : "v"(u[i])); asm volatile("" : "+v"(d[i]), "+v"(u[i]));
#define MOV64(i) asm volatile("v_mov_b64 %0, %0" : "+v"(d[i]));
#define CMP(i) asm volatile("v_cmp_lt_f64 vcc, %0, %0" :: "v"(d[i]) : "vcc");
#define CND(i) asm volatile("v_cndmask_b32 %0, %0, %0, vcc" : "+v"(u[i]) :: "vcc");
        if (K == 0) { BODY8(FMA) }
        if (K == 1) { BODY8(MUL) }
        if (K == 2) { BODY8(ADD) }
        if (K == 3) { BODY8(RCP) }
        if (K == 4) { BODY8(RSQ) }
        if (K == 5) { BODY8(DSC) }
        if (K == 6) { BODY8(DFX) }
        if (K == 7) { BODY8(MAD64) }
        if (K == 8) { BODY8(MULLO) }
        if (K == 9) { BODY8(MULHI) }
        if (K == 10) { BODY8(M24) }
        if (K == 11) { BODY8(IADD) }
        if (K == 12) { BODY8(CVT) }
        if (K == 13) { BODY8(MOV64) }
        if (K == 14) { BODY8(CMP) }
        if (K == 15) { BODY8(CND) }
#define FADD(i) asm volatile("v_add_f32 %0, %0, %0" : "+v"(f[i]));
#define FFMA(i) asm volatile("v_fma_f32 %0, %0, %0, %0" : "+v"(f[i]));
#define PKFMA(i) asm volatile("v_pk_fma_f32 %0, %0, %0, %0" : "+v"(d[i]));
#define FMIN3(i) asm volatile("v_min3_f32 %0, %0, %0, %0" : "+v"(f[i]));
#define DMIN(i) asm volatile("v_min_f64 %0, %0, %0" : "+v"(d[i]));
#define CVTF(i) asm volatile("v_cvt_f32_f64 %0, %1" : "=v"(f[i]) : "v"(d[i])); asm volatile("" : "+v"(f[i]), "+v"(d[i]));
        if (K == 16) { BODY8(FADD) }
        if (K == 17) { BODY8(FFMA) }
        if (K == 18) { BODY8(PKFMA) }
        if (K == 19) { BODY8(FMIN3) }
        if (K == 20) { BODY8(DMIN) }
        if (K == 21) { BODY8(CVTF) }
#define FRCP(i) asm volatile("v_rcp_f32 %0, %0" : "+v"(f[i]));
#define FSQRT(i) asm volatile("v_sqrt_f32 %0, %0" : "+v"(f[i]));
#define FEXP(i) asm volatile("v_exp_f32 %0, %0" : "+v"(f[i]));
#define FSIN(i) asm volatile("v_sin_f32 %0, %0" : "+v"(f[i]));
#define MOV32(i) asm volatile("v_mov_b32 %0, %0" : "+v"(u[i]));
#define FCMP(i) asm volatile("v_cmp_lt_f32 s[40:41], %0, %0" :: "v"(f[i]) : "s40", "s41");
#define CNDS(i) asm volatile("v_cndmask_b32 %0, %0, %0, s[42:43]" : "+v"(u[i]) :: "s42", "s43");
#define AND32(i) asm volatile("v_and_b32 %0, %0, %0" : "+v"(u[i]));
#define LSHL(i) asm volatile("v_lshlrev_b32 %0, 3, %0" : "+v"(u[i]));
#define DSQRT(i) asm volatile("v_sqrt_f64 %0, %0" : "+v"(d[i]));
#define PKMUL(i) asm volatile("v_pk_mul_f32 %0, %0, %0" : "+v"(d[i]));
#define BFE(i) asm volatile("v_bfe_u32 %0, %0, 3, 7" : "+v"(u[i]));
        if (K == 22) { BODY8(FRCP) }
        if (K == 23) { BODY8(FSQRT) }
        if (K == 24) { BODY8(FEXP) }
        if (K == 25) { BODY8(FSIN) }
        if (K == 26) { BODY8(MOV32) }
        if (K == 27) { BODY8(FCMP) }
        if (K == 28) { BODY8(CNDS) }
        if (K == 29) { BODY8(AND32) }
        if (K == 30) { BODY8(LSHL) }
        if (K == 31) { BODY8(DSQRT) }
        if (K == 32) { BODY8(PKMUL) }
        if (K == 33) { BODY8(BFE) }
#define FMIX(i) asm volatile("v_fma_mix_f32 %0, %0, %0, %0 op_sel_hi:[1,0,0]" : "+v"(f[i]));
#define CVTH(i) asm volatile("v_cvt_f32_f16 %0, %0" : "+v"(f[i]));
        if (K == 34) { BODY8(FMIX) }
        if (K == 35) { BODY8(CVTH) }
    }
    double s = 0;
    for (int i = 0; i < 8; ++i) s += d[i] + (double)u[i] + (double)w[i] + (double)f[i];
    if (s == 12345.678) out[threadIdx.x] = s;
}

static const char* kNames[] = {"v_fma_f64", "v_mul_f64", "v_add_f64", "v_rcp_f64", "v_rsq_f64", "v_div_scale_f64",
                               "v_div_fixup_f64", "v_mad_u64_u32", "v_mul_lo_u32", "v_mul_hi_u32",
                               "v_mul_u32_u24", "v_add_u32", "v_cvt_f64_u32", "v_mov_b64", "v_cmp_lt_f64",
                               "v_cndmask_b32", "v_add_f32", "v_fma_f32", "v_pk_fma_f32",
                               "v_min3_f32", "v_min_f64", "v_cvt_f32_f64", "v_rcp_f32", "v_sqrt_f32",
                               "v_exp_f32", "v_sin_f32", "v_mov_b32", "v_cmp_lt_f32", "v_cndmask_b32 (sgpr)",
                               "v_and_b32", "v_lshlrev_b32", "v_sqrt_f64", "v_pk_mul_f32", "v_bfe_u32",
                               "v_fma_mix_f32", "v_cvt_f32_f16"};

template <int K>
static int run(double* out, int cus, double clk_ghz) {
    const int blocks = cus * 4;  // 4 blocks x 4 waves per CU = 4 waves per SIMD
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    hipLaunchKernelGGL(k_rate<K>, dim3(blocks), dim3(256), 0, 0, out, 1u);
    CHK(hipEventRecord(a));
    hipLaunchKernelGGL(k_rate<K>, dim3(blocks), dim3(256), 0, 0, out, 2u);
    CHK(hipEventRecord(b));
    CHK(hipEventSynchronize(b));
    float ms;
    CHK(hipEventElapsedTime(&ms, a, b));
    // wave-instructions per SIMD: 4 waves x iters x 8
    const double per_simd = 4.0 * kIters * 8;
    const double cycles = ms * 1e-3 * clk_ghz * 1e9;
    std::printf("%-18s %7.3f ms  %5.2f cycles per wave-instruction per SIMD\n", kNames[K], ms, cycles / per_simd);
    return 0;
}

int main() {
    hipDeviceProp_t p;
    CHK(hipGetDeviceProperties(&p, 0));
    const double clk = p.clockRate * 1e-6;  // kHz -> GHz
    std::printf("%s, %d CUs, clock %.2f GHz (nominal)\n", p.gcnArchName, p.multiProcessorCount, clk);
    double* out;
    CHK(hipMalloc(&out, 256 * sizeof(double)));
    run<0>(out, p.multiProcessorCount, clk); run<1>(out, p.multiProcessorCount, clk);
    run<2>(out, p.multiProcessorCount, clk); run<3>(out, p.multiProcessorCount, clk);
    run<4>(out, p.multiProcessorCount, clk); run<5>(out, p.multiProcessorCount, clk);
    run<6>(out, p.multiProcessorCount, clk); run<7>(out, p.multiProcessorCount, clk);
    run<8>(out, p.multiProcessorCount, clk); run<9>(out, p.multiProcessorCount, clk);
    run<10>(out, p.multiProcessorCount, clk); run<11>(out, p.multiProcessorCount, clk);
    run<12>(out, p.multiProcessorCount, clk); run<13>(out, p.multiProcessorCount, clk);
    run<14>(out, p.multiProcessorCount, clk); run<15>(out, p.multiProcessorCount, clk);
    run<16>(out, p.multiProcessorCount, clk); run<17>(out, p.multiProcessorCount, clk);
    run<18>(out, p.multiProcessorCount, clk); run<19>(out, p.multiProcessorCount, clk);
    run<20>(out, p.multiProcessorCount, clk); run<21>(out, p.multiProcessorCount, clk);
    run<22>(out, p.multiProcessorCount, clk); run<23>(out, p.multiProcessorCount, clk);
    run<24>(out, p.multiProcessorCount, clk); run<25>(out, p.multiProcessorCount, clk);
    run<26>(out, p.multiProcessorCount, clk); run<27>(out, p.multiProcessorCount, clk);
    run<28>(out, p.multiProcessorCount, clk); run<29>(out, p.multiProcessorCount, clk);
    run<30>(out, p.multiProcessorCount, clk); run<31>(out, p.multiProcessorCount, clk);
    run<32>(out, p.multiProcessorCount, clk); run<33>(out, p.multiProcessorCount, clk);
    run<34>(out, p.multiProcessorCount, clk); run<35>(out, p.multiProcessorCount, clk);
    CHK(hipFree(out));
    return 0;
}
