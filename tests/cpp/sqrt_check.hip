// sqrt_check.hip — on the card: rtw_div.h's sqrt_core(x) is bit-identical to
// the compiler's sqrt(x) for positive finite x >= 2^-766 (sqrt_core_ok), and
// sqrt_w equals it everywhere, zeros, subnormals, infinities, negatives and
// NaNs included.  Test tool (tests/test_div_hw.py).
//
//   sqrt_check <log2 samples per class>   prints "class <k> mismatches <n> of <m>"
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
__device__ __forceinline__ double from_bits(unsigned long long b) {
    double v;
    memcpy(&v, &b, 8);
    return v;
}
__device__ __forceinline__ unsigned long long bits_of(double v) {
    unsigned long long b;
    memcpy(&b, &v, 8);
    return b;
}

__global__ void k_check(int cls, unsigned long long n, unsigned long long* bad) {
    unsigned long long local = 0;
    for (unsigned long long i = blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x; i < n;
         i += (unsigned long long)gridDim.x * blockDim.x) {
        const unsigned long long r = mix(i * 3 + (unsigned long long)cls * 0x1000000000ull);
        double x;
        if (cls == 0) {  // the core's whole range: exponent field 257..2046, any mantissa
            x = from_bits(((257ull + (r >> 52) % 1790ull) << 52) | (r & 0xFFFFFFFFFFFFFull));
        } else if (cls == 1) {  // the kernels' values: [0, 4) (1 - r2, r2, discriminants, lengths^2)
            x = (double)(r >> 11) * 0x1p-51;
        } else if (cls == 2) {  // the range's low edge (2^-766 ...) and around 1
            const unsigned long long e = (r >> 60) & 1 ? 257ull + (r >> 52) % 16ull : 1018ull + (r >> 52) % 10ull;
            x = from_bits((e << 52) | (r & 0xFFFFFFFFFFFFFull));
        } else {  // anything at all (sqrt_w only): all bit patterns, with zeros, infinities and the
                  // doubles just below the core's range (2^-774 .. 2^-766) mixed in
            const unsigned long long k = r & 15;
            x = k == 0   ? 0.0
                : k == 1 ? -0.0
                : k == 2 ? __builtin_inf()
                : k == 3 ? -1.0
                : k == 4 ? from_bits(((249ull + (r >> 52) % 8ull) << 52) | (r & 0xFFFFFFFFFFFFFull))
                         : from_bits(r);
        }
        const double want = __builtin_sqrt(x);
        const double w = rtwd::sqrt_w(x);
        bool ok = bits_of(w) == bits_of(want) || (want != want && w != w);
        if (cls < 3) ok = ok && rtwd::sqrt_core_ok(x) && bits_of(rtwd::sqrt_core(x)) == bits_of(want);
        local += !ok;
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
