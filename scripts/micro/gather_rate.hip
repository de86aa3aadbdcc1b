// Microbenchmark: throughput of 64-lane buffer_load_dwordx2 gathers from L2-resident data (gfx950) for
// lane-address patterns like k_eval_nb's texel fetches.  A pattern is `runs` runs of `g` lanes; lanes of
// a run are `in` bytes apart, runs `out` bytes apart.  Every iteration moves the whole pattern by a
// large odd offset inside a 2 MB buffer (L2-resident, mostly L1 misses).  Prints cycles per wave
// instruction per CU at the measured clock-free rate (ns per instruction per CU x 2.4 GHz).
#include <hip/hip_runtime.h>
#include <cstdio>

typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// W = 8 or 16 bytes per lane; step = the pattern's move per iteration (69632: L1 misses; 8: the next
// iteration touches the same lines, as consecutive samples of one lane mostly do)
template <int W>
__global__ __launch_bounds__(256) void k_gather(const unsigned* buf, unsigned* out, int g, int in, int out_stride,
                                                int iters, unsigned bytes, unsigned step) {
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned*>(buf), 0, bytes, 0x00020000);
    const int lane = threadIdx.x & 63;
    const unsigned base = (lane % g) * in + (lane / g) * out_stride + (blockIdx.x * 4 + threadIdx.x / 64) * 8192u;
    unsigned acc = 0;
    const unsigned mask = (bytes - 1) & ~7u;   // bytes: power of two
    for (int i = 0; i < iters; i += 4) {
        if (W == 8) {
            u32x2 v[4];
#pragma unroll
            for (int k = 0; k < 4; ++k)
                v[k] = __builtin_amdgcn_raw_buffer_load_b64(rs, (base + (i + k) * step) & mask, 0, 0);
#pragma unroll
            for (int k = 0; k < 4; ++k) acc ^= v[k].x + v[k].y;
        } else {
            u32x4 v[4];
#pragma unroll
            for (int k = 0; k < 4; ++k)
                v[k] = __builtin_amdgcn_raw_buffer_load_b128(rs, (base + (i + k) * step) & mask & ~15u, 0, 0);
#pragma unroll
            for (int k = 0; k < 4; ++k) acc ^= v[k].x + v[k].y + v[k].z + v[k].w;
        }
    }
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

int main() {
    const unsigned bytes = 2u << 20;
    const int blocks = 256 * 8, iters = 2048;
    unsigned *buf, *out;
    (void)hipMalloc(&buf, bytes);
    (void)hipMemset(buf, 1, bytes);
    (void)hipMalloc(&out, sizeof(unsigned) * blocks * 256);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    struct P { const char* name; int g, in, out; } pats[] = {
        {"64 lanes contiguous (512 B, 4 lines)", 64, 8, 0},
        {"8 runs x 8 lanes, 8 B apart (8 x 64 B)", 8, 8, 4096},
        {"8 runs x 8 lanes, 16 B apart (8 x 128 B)", 8, 16, 4096},
        {"16 runs x 4 lanes, 8 B apart", 4, 8, 4096},
        {"32 runs x 2 lanes, 8 B apart", 2, 8, 4096},
        {"64 lanes, one line each (256 B apart)", 1, 0, 256},
        {"64 lanes, one line each (4160 B apart)", 1, 0, 4160},
        {"8 runs x 8 lanes, 24 B apart (k_eval_nb-like)", 8, 24, 4160},
    };
    const unsigned steps[2] = {69632u, 8u};
    for (int st = 0; st < 2; ++st)
        for (int w = 8; w <= 16; w += 8)
            for (const P& p : pats)
                for (int rep = 0; rep < 2; ++rep) {
                    auto launch = [&]() {
                        if (w == 8) k_gather<8><<<blocks, 256>>>(buf, out, p.g, p.in, p.out, iters, bytes, steps[st]);
                        else k_gather<16><<<blocks, 256>>>(buf, out, p.g, p.in, p.out, iters, bytes, steps[st]);
                    };
                    launch();
                    (void)hipEventRecord(e0);
                    launch();
                    (void)hipEventRecord(e1);
                    (void)hipEventSynchronize(e1);
                    float ms = 0.f;
                    (void)hipEventElapsedTime(&ms, e0, e1);
                    const double instr_per_cu = double(blocks) * 4 * iters / 256.0;
                    const double ns = ms * 1e6 / instr_per_cu;
                    if (rep == 1)
                        printf("step %5u  %2d B/lane  %-48s %6.2f ns/instr/CU  %6.1f cycles@2.4GHz\n", steps[st], w, p.name,
                               ns, ns * 2.4);
                }
    return 0;
}
