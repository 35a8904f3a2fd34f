// Microbenchmark: a hub-row fma chain fed from a pre-staged contiguous panel in global memory
// (Z[group of 4 links][d columns][4]) with global_load_dwordx4, values through scalar loads --
// against the LDS-fed consumer of k_spmm_hub (tools/probes/lds_chain.hip).  Prints cycles per link
// (s_memtime = shader cycles) and the wall time of one launch.
//   hipcc -O3 --offload-arch=gfx950 tools/probes/hub_stream.hip -o /tmp/hub_stream && /tmp/hub_stream
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <vector>
typedef float V4 __attribute__((ext_vector_type(4)));

// one wave per (row, column block of COLS); lanes >= COLS idle.  VALS: 0 constant, 1 scalar loads
template <int COLS, int R, int VALS, int BUF = 0>
__global__ void __launch_bounds__(64) k_chain(const float* __restrict__ Z, const float* __restrict__ vals, int n_links,
                                              int d, float* __restrict__ out, long long* __restrict__ cyc, int reps)
{
    const int lane = threadIdx.x;
    const int c0 = blockIdx.x * COLS;
    const int ng = n_links >> 2;                       // groups (n_links % (4R) == 0 here)
    const uint32_t loff = (uint32_t)(c0 + lane) * 16u;   // lane offset (bytes) inside a group
    const size_t gstride = (size_t)d * 16;                 // bytes per 4-link group
    float acc = 0.f;
    long long t0 = __builtin_amdgcn_s_memtime();
    if (lane < COLS) {
        for (int rep = 0; rep < reps; ++rep) {
            V4 buf[R];
            const char* zb = reinterpret_cast<const char*>(Z);
            const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(Z), 0, 0x7fffffff, 0x00020000);
#pragma unroll
            for (int i = 0; i < R; ++i)
                buf[i] = __builtin_nontemporal_load(reinterpret_cast<const V4*>(zb + i * gstride + loff));
            for (int g = 0; g < ng; g += R) {
                const char* zn = zb + (size_t)(g + R) * gstride;   // wave-uniform (Z padded by R groups)
                const float* av = vals + 4 * g;
#pragma unroll
                for (int i = 0; i < R; ++i) {
                    float a0, a1, a2, a3;
                    if (VALS) {
                        a0 = av[4 * i]; a1 = av[4 * i + 1]; a2 = av[4 * i + 2]; a3 = av[4 * i + 3];
                    } else {
                        a0 = 0.5f; a1 = 0.25f; a2 = 0.125f; a3 = 0.75f;
                    }
                    acc = __builtin_fmaf(a0, buf[i][0], acc);
                    acc = __builtin_fmaf(a1, buf[i][1], acc);
                    acc = __builtin_fmaf(a2, buf[i][2], acc);
                    acc = __builtin_fmaf(a3, buf[i][3], acc);
                    if (BUF)
                        buf[i] = __builtin_bit_cast(V4, __builtin_amdgcn_raw_buffer_load_b128(
                            rsrc, loff, (uint32_t)((g + R + i) * gstride), 0));
                    else
                        buf[i] = __builtin_nontemporal_load(reinterpret_cast<const V4*>(zn + i * gstride + loff));
                }
            }
        }
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) cyc[blockIdx.x] = t1 - t0;
    if (lane < COLS) out[c0 + lane] = acc;
}

template <int COLS, int R, int VALS, int BUF = 0>
void run(const char* name, const float* Z, const float* vals, int n_links, int d, float* out, long long* cyc, int reps)
{
    const int blocks = d / COLS;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    hipLaunchKernelGGL((k_chain<COLS, R, VALS, BUF>), dim3(blocks), dim3(64), 0, 0, Z, vals, n_links, d, out, cyc, reps);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL((k_chain<COLS, R, VALS, BUF>), dim3(blocks), dim3(64), 0, 0, Z, vals, n_links, d, out, cyc, reps);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    std::vector<long long> c(blocks);
    (void)hipMemcpy(c.data(), cyc, 8 * blocks, hipMemcpyDeviceToHost);
    long long mx = 0;
    for (auto v : c) mx = v > mx ? v : mx;
    const double links = (double)n_links * reps;
    printf("%-34s links=%9d reps=%3d blocks=%d  %.2f cycles/link  %.3f ms  (%.2f ns/link)\n", name, n_links, reps,
           blocks, (double)mx / links, ms, ms * 1e6 / links);
}

int main()
{
    const int d = 128;
    const int big = 155904;                 // the products top hub row (155,868) rounded up to 64
    float *Z, *vals, *out;
    long long* cyc;
    (void)hipMalloc(&Z, (size_t)(big + 4 * 64) * d * 4);   // + R groups of padding
    (void)hipMalloc(&vals, (size_t)big * 4);
    (void)hipMalloc(&out, d * 4);
    (void)hipMalloc(&cyc, 8 * 64);
    {
        std::vector<float> h((size_t)big * d);
        for (size_t i = 0; i < h.size(); ++i) h[i] = (float)((i * 2654435761u) % 1000) * 1e-3f - 0.5f;
        (void)hipMemcpy(Z, h.data(), h.size() * 4, hipMemcpyHostToDevice);
        (void)hipMemcpy(vals, h.data(), (size_t)big * 4, hipMemcpyHostToDevice);
    }
    // L2-resident stream (4096 links = 2 MB at d=128), repeated
    run<64, 16, 0>("warm 64 cols R16 const vals", Z, vals, 4096, d, out, cyc, 40);
    run<64, 16, 1>("warm 64 cols R16 scalar vals", Z, vals, 4096, d, out, cyc, 40);
    run<32, 16, 1>("warm 32 cols R16 scalar vals", Z, vals, 4096, d, out, cyc, 40);
    run<64, 32, 1>("warm 64 cols R32 scalar vals", Z, vals, 4096, d, out, cyc, 40);
    // the top hub row streamed once (80 MB)
    run<64, 16, 1>("hub 64 cols R16 scalar vals", Z, vals, big, d, out, cyc, 1);
    run<64, 32, 1>("hub 64 cols R32 scalar vals", Z, vals, big, d, out, cyc, 1);
    run<32, 16, 1>("hub 32 cols R16 scalar vals", Z, vals, big, d, out, cyc, 1);
    run<32, 32, 1>("hub 32 cols R32 scalar vals", Z, vals, big, d, out, cyc, 1);
    run<16, 32, 1>("hub 16 cols R32 scalar vals", Z, vals, big, d, out, cyc, 1);
    run<64, 16, 0>("hub 64 cols R16 const vals", Z, vals, big, d, out, cyc, 1);
    run<64, 16, 1, 1>("warm 64 cols R16 scalar vals buf", Z, vals, 4096, d, out, cyc, 40);
    run<32, 16, 1, 1>("warm 32 cols R16 scalar vals buf", Z, vals, 4096, d, out, cyc, 40);
    run<64, 16, 1, 1>("hub 64 cols R16 scalar vals buf", Z, vals, big, d, out, cyc, 1);
    run<64, 32, 1, 1>("hub 64 cols R32 scalar vals buf", Z, vals, big, d, out, cyc, 1);
    run<32, 32, 1, 1>("hub 32 cols R32 scalar vals buf", Z, vals, big, d, out, cyc, 1);
    run<16, 32, 1, 1>("hub 16 cols R32 scalar vals buf", Z, vals, big, d, out, cyc, 1);
    return 0;
}
