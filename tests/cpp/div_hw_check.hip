// div_hw_check.hip — on the card: rtw_div.h's shared-divisor quotient
// div_hw(a, b, rcp_hw(b)) is bit-identical to the compiler's a / b for
// |b| in [2^-200, 2^200], |a| in [2^-800, 2^100] (random exponents and
// mantissas over the whole range, plus the value ranges the kernels see:
// scene coordinates over ray-direction components, vector lengths, pdfs),
// and both quotients of a smaller |a| stay below 2^-599 in magnitude (what
// the ray tests rely on to reject them alike).  Test tool (tests/test_div_hw.py).
//
//   div_hw_check <log2 samples per class>   prints "class <k> mismatches <n> of <m>"
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include "rtw_div.h"

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { std::printf("HIP error %s\n", hipGetErrorString(e)); return 2; } } while (0)

__device__ __forceinline__ unsigned long long mix(unsigned long long x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
// random double with exponent uniform in [elo, ehi) (so |v| in [2^elo, 2^ehi)), random mantissa and sign
__device__ __forceinline__ double rnd_exp(unsigned long long r, int elo, int ehi) {
    const int e = elo + (int)((r >> 53) % (unsigned long long)(ehi - elo));
    const unsigned long long bits = ((unsigned long long)(e + 1023) << 52) | (r & 0xFFFFFFFFFFFFFull);
    double v;
    memcpy(&v, &bits, 8);
    return ((r >> 52) & 1) ? -v : v;
}
__device__ __forceinline__ double u01(unsigned long long r) { return (double)(r >> 11) * 0x1p-53; }

__global__ void k_check(int cls, unsigned long long n, unsigned long long* bad) {
    unsigned long long local = 0;
    for (unsigned long long i = blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x; i < n;
         i += (unsigned long long)gridDim.x * blockDim.x) {
        const unsigned long long r1 = mix(i * 2 + (unsigned long long)cls * 0x1000000000ull), r2 = mix(r1 ^ 0x5555);
        double a, b;
        if (cls == 0) {  // whole guarded range
            a = rnd_exp(r1, -800, 100);
            b = rnd_exp(r2, -200, 200);
        } else if (cls == 1) {  // scene coordinate differences over direction components
            a = (u01(r1) - 0.5) * 2000.0;
            b = (u01(r2) - 0.5) * 2.0;
        } else if (cls == 2) {  // components over a length / pdf-sized divisors
            a = (u01(r1) - 0.5) * 2.0;
            b = 1e-3 + u01(r2) * 1e3;
        } else {  // |a| below the range (incl. zeros and subnormals): both tiny
            a = (r1 & 7) == 0 ? ((r1 & 8) ? -0.0 : 0.0) : rnd_exp(r1, -1022, -800) * ((r1 & 16) ? 0x1p-52 : 1.0);
            b = rnd_exp(r2, -200, 200);
        }
        if (!rtwd::div_hw_ok_b(b)) { ++local; continue; }  // the generator must stay in range
        const double want = a / b;
        const double got = rtwd::div_hw(a, b, rtwd::rcp_hw(b));
        if (cls < 3) {
            if (!rtwd::div_hw_ok_a(a)) { ++local; continue; }
            unsigned long long wb, gb;
            memcpy(&wb, &want, 8);
            memcpy(&gb, &got, 8);
            local += wb != gb;
        } else {
            local += !(__builtin_fabs(want) < 0x1p-599 && __builtin_fabs(got) < 0x1p-599);
        }
    }
    if (local) atomicAdd(bad, local);
}

int main(int argc, char** argv) {
    const int lg = argc > 1 ? std::atoi(argv[1]) : 28;
    const unsigned long long n = 1ull << lg;
    unsigned long long* bad;
    CHK(hipMalloc(&bad, sizeof(unsigned long long)));
    int fails = 0;
    for (int cls = 0; cls < 4; ++cls) {
        CHK(hipMemset(bad, 0, sizeof(unsigned long long)));
        hipLaunchKernelGGL(k_check, dim3(4096), dim3(256), 0, 0, cls, n, bad);
        CHK(hipGetLastError());
        unsigned long long h = 0;
        CHK(hipMemcpy(&h, bad, sizeof h, hipMemcpyDeviceToHost));
        std::printf("class %d mismatches %llu of %llu\n", cls, h, n);
        fails += h != 0;
    }
    CHK(hipFree(bad));
    return fails ? 1 : 0;
}
