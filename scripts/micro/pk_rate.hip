// Microbenchmark: issue rate of v_fma_f32 vs v_pk_fma_f32 (wave64, gfx950).  Each lane runs 8
// independent accumulator chains; one launch fills every SIMD with 8 waves.  Prints TFLOP/s (FMA = 2).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f2 __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(256) void k_scalar(float* out, float a, float b, int iters) {
    float x[8];
    for (int k = 0; k < 8; ++k) x[k] = threadIdx.x * 1e-3f + k;
    for (int i = 0; i < iters; ++i)
#pragma unroll
        for (int k = 0; k < 8; ++k) x[k] = fmaf(x[k], a, b);
    float s = 0.f;
    for (int k = 0; k < 8; ++k) s += x[k];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_packed(float* out, float a, float b, int iters) {
    f2 x[4];
    for (int k = 0; k < 4; ++k) x[k] = (f2){threadIdx.x * 1e-3f + k, threadIdx.x * 2e-3f + k};
    const f2 av = (f2)(a), bv = (f2)(b);
    for (int i = 0; i < iters; ++i)
#pragma unroll
        for (int k = 0; k < 4; ++k) x[k] = __builtin_elementwise_fma(x[k], av, bv);
    float s = 0.f;
    for (int k = 0; k < 4; ++k) s += x[k].x + x[k].y;
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

int main() {
    const int blocks = 256 * 8 * 4, iters = 4096;
    float* out;
    (void)hipMalloc(&out, sizeof(float) * blocks * 256);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int rep = 0; rep < 3; ++rep) {
        for (int m = 0; m < 2; ++m) {
            (void)hipEventRecord(e0);
            if (m == 0) k_scalar<<<blocks, 256>>>(out, 0.999f, 1e-3f, iters);
            else k_packed<<<blocks, 256>>>(out, 0.999f, 1e-3f, iters);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms;
            (void)hipEventElapsedTime(&ms, e0, e1);
            const double flop = 2.0 * 8 * iters * double(blocks) * 256;
            std::printf("%s: %.3f ms, %.1f TFLOP/s\n", m ? "v_pk_fma_f32" : "v_fma_f32   ", ms, flop / ms / 1e9);
        }
    }
    (void)hipFree(out);
    return 0;
}
