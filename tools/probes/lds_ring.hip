// Microbenchmark: the hub consumer's chain (one fma per link per lane, lane = column) fed by
// ds_read_b128 tile reads with a ring of L reads in flight, and the link values from
//   VAL 0: constants, 1: LDS (broadcast ds_read_b128), 2: global (broadcast global_load_dwordx4).
// Optionally next to 8 waves writing LDS (the producers' traffic).  Prints shader cycles per link.
//   hipcc -O3 --offload-arch=gfx950 tools/probes/lds_ring.hip -o /tmp/lds_ring && /tmp/lds_ring
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float V4 __attribute__((ext_vector_type(4)));
constexpr int LD = 528, W = 512, NG = W / 4;   // tile [32 cols][LD], 128 groups of 4 links

template <int L, int VAL>
__global__ void __launch_bounds__(576) k(const float* __restrict__ gvals, float* out, long long* cyc, int reps,
                                         int busy, int active)
{
    __shared__ __attribute__((aligned(16))) float lds[32 * LD + W];
    for (int i = threadIdx.x; i < 32 * LD + W; i += blockDim.x) lds[i] = (float)(i % 97) * 0.01f;
    __syncthreads();
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (wave != 0) {
        if (busy) {
            float x = lane;
            for (int r = 0; r < reps * 16; ++r) lds[(lane * 33 + r * 64 + wave) % (32 * LD)] = x;
        }
        return;
    }
    const int c = lane & 31, sw = (c >> 2) & 7;
    const float* tcol = lds + c * LD;
    const float* av = lds + 32 * LD;
    float acc = 0.f;
    long long t0 = __builtin_amdgcn_s_memtime();
    if (lane < active) {
        int vz;   // an opaque per-lane zero: keeps the value loads on the vector path
        asm volatile("v_mov_b32 %0, 0" : "=v"(vz));
        const V4* gv4 = reinterpret_cast<const V4*>(gvals) + vz;
#pragma nounroll
        for (int r = 0; r < reps; ++r) {
            V4 t[L], a[L];
#pragma unroll
            for (int i = 0; i < L; ++i) {
                t[i] = *reinterpret_cast<const V4*>(tcol + ((i ^ sw) << 2));
                if (VAL == 1) a[i] = *reinterpret_cast<const V4*>(av + (i << 2));
                if (VAL == 2) a[i] = __builtin_nontemporal_load(gv4 + i);
            }
#pragma nounroll
            for (int g = 0; g < NG; g += L) {
#pragma unroll
                for (int i = 0; i < L; ++i) {
                    V4 aa = VAL == 0 ? V4{0.5f, 0.25f, 0.125f, 0.75f} : a[i];
                    acc = __builtin_fmaf(aa[0], t[i][0], acc);
                    acc = __builtin_fmaf(aa[1], t[i][1], acc);
                    acc = __builtin_fmaf(aa[2], t[i][2], acc);
                    acc = __builtin_fmaf(aa[3], t[i][3], acc);
                    const int gn = (g + L + i) & (NG - 1);
                    t[i] = *reinterpret_cast<const V4*>(tcol + ((gn ^ sw) << 2));
                    if (VAL == 1) a[i] = *reinterpret_cast<const V4*>(av + (gn << 2));
                    if (VAL == 2) a[i] = __builtin_nontemporal_load(gv4 + gn);
                }
            }
        }
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) cyc[blockIdx.x] = t1 - t0;
    out[threadIdx.x] = acc;
}

template <int L, int VAL>
void run(const float* gv, float* out, long long* cyc, int busy, int active)
{
    const int reps = 200;
    hipLaunchKernelGGL((k<L, VAL>), dim3(1), dim3(576), 0, 0, gv, out, cyc, reps, busy, active);
    (void)hipDeviceSynchronize();
    long long c;
    (void)hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    const int groups = ((NG + L - 1) / L) * L;
    printf("L=%2d val=%-6s busy=%d active=%2d  %.2f cycles/link\n", L, VAL == 0 ? "const" : VAL == 1 ? "lds" : "global",
           busy, active, (double)c / ((double)reps * groups * 4));
}


// the same chain with the window fully unrolled: tile reads at per-lane bases b[k] (k = group & 7,
// the XOR swizzle folded in) + immediate offsets, value reads at one base + immediate offsets
template <int L, int VAL>
__global__ void __launch_bounds__(576) k_imm(const float* __restrict__ gvals, float* out, long long* cyc, int reps,
                                             int busy, int active)
{
    __shared__ __attribute__((aligned(16))) float lds[32 * LD + W];
    for (int i = threadIdx.x; i < 32 * LD + W; i += blockDim.x) lds[i] = (float)(i % 97) * 0.01f;
    __syncthreads();
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (wave != 0) {
        if (busy) {
            float x = lane;
            for (int r = 0; r < reps * 16; ++r) lds[(lane * 33 + r * 64 + wave) % (32 * LD)] = x;
        }
        return;
    }
    const int c = lane & 31, sw = (c >> 2) & 7;
    const float* b[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) b[k] = lds + c * LD + ((k ^ sw) << 2);
    const float* av = lds + 32 * LD;
    int vz;
    asm volatile("v_mov_b32 %0, 0" : "=v"(vz));
    const V4* gv4 = reinterpret_cast<const V4*>(gvals) + vz;
    float acc = 0.f;
    long long t0 = __builtin_amdgcn_s_memtime();
    if (lane < active) {
#pragma nounroll
        for (int r = 0; r < reps; ++r) {
            V4 t[L], a[L];
#pragma unroll
            for (int i = 0; i < L; ++i) {
                t[i] = *reinterpret_cast<const V4*>(b[i & 7] + (i >> 3) * 32);
                if (VAL == 1) a[i] = *reinterpret_cast<const V4*>(av + (i << 2));
                if (VAL == 2) a[i] = __builtin_nontemporal_load(gv4 + i);
            }
#pragma unroll
            for (int g0 = 0; g0 < NG; g0 += L) {
#pragma unroll
                for (int i = 0; i < L; ++i) {
                    const int g = g0 + i;
                    if (g < NG) {
                        V4 aa = VAL == 0 ? V4{0.5f, 0.25f, 0.125f, 0.75f} : a[i];
                        acc = __builtin_fmaf(aa[0], t[i][0], acc);
                        acc = __builtin_fmaf(aa[1], t[i][1], acc);
                        acc = __builtin_fmaf(aa[2], t[i][2], acc);
                        acc = __builtin_fmaf(aa[3], t[i][3], acc);
                        const int gn = g + L;
                        if (gn < NG) {
                            t[i] = *reinterpret_cast<const V4*>(b[gn & 7] + (gn >> 3) * 32);
                            if (VAL == 1) a[i] = *reinterpret_cast<const V4*>(av + (gn << 2));
                            if (VAL == 2) a[i] = __builtin_nontemporal_load(gv4 + gn);
                        }
                        __builtin_amdgcn_sched_barrier(0);
                    }
                }
            }
        }
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) cyc[blockIdx.x] = t1 - t0;
    out[threadIdx.x] = acc;
}

template <int L, int VAL>
__global__ void __launch_bounds__(576) k_bar(const float* __restrict__ gvals, float* out, long long* cyc, int reps,
                                             int busy, int active)
{
    __shared__ __attribute__((aligned(16))) float lds[32 * LD + W];
    for (int i = threadIdx.x; i < 32 * LD + W; i += blockDim.x) lds[i] = (float)(i % 97) * 0.01f;
    __syncthreads();
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (wave != 0) {
        for (int r = 0; r < reps; ++r) __syncthreads();
        return;
    }
    const int c = lane & 31, sw = (c >> 2) & 7;
    const float* b[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) b[k] = lds + c * LD + ((k ^ sw) << 2);
    const float* av = lds + 32 * LD;
    int vz;
    asm volatile("v_mov_b32 %0, 0" : "=v"(vz));
    const V4* gv4 = reinterpret_cast<const V4*>(gvals) + vz;
    float acc = 0.f;
    long long t0 = __builtin_amdgcn_s_memtime();
#pragma nounroll
    for (int r = 0; r < reps; ++r) {
        __syncthreads();
        if (lane < active) {
            V4 t[L], a[L];
#pragma unroll
            for (int i = 0; i < L; ++i) {
                t[i] = *reinterpret_cast<const V4*>(b[i & 7] + (i >> 3) * 32);
                if (VAL == 1) a[i] = *reinterpret_cast<const V4*>(av + (i << 2));
                if (VAL == 2) a[i] = __builtin_nontemporal_load(gv4 + i);
            }
#pragma unroll
            for (int g0 = 0; g0 < NG; g0 += L) {
#pragma unroll
                for (int i = 0; i < L; ++i) {
                    const int g = g0 + i;
                    if (g < NG) {
                        V4 aa = VAL == 0 ? V4{0.5f, 0.25f, 0.125f, 0.75f} : a[i];
                        acc = __builtin_fmaf(aa[0], t[i][0], acc);
                        acc = __builtin_fmaf(aa[1], t[i][1], acc);
                        acc = __builtin_fmaf(aa[2], t[i][2], acc);
                        acc = __builtin_fmaf(aa[3], t[i][3], acc);
                        const int gn = g + L;
                        if (gn < NG) {
                            t[i] = *reinterpret_cast<const V4*>(b[gn & 7] + (gn >> 3) * 32);
                            if (VAL == 1) a[i] = *reinterpret_cast<const V4*>(av + (gn << 2));
                            if (VAL == 2) a[i] = __builtin_nontemporal_load(gv4 + gn);
                        }
                        __builtin_amdgcn_sched_barrier(0);
                    }
                }
            }
        }
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) cyc[blockIdx.x] = t1 - t0;
    out[threadIdx.x] = acc;
}

template <int L, int VAL>
void run_imm(const float* gv, float* out, long long* cyc, int busy, int active, bool bar = false)
{
    const int reps = 200;
    auto fn = bar ? k_bar<L, VAL> : k_imm<L, VAL>;
    hipLaunchKernelGGL(fn, dim3(1), dim3(576), 0, 0, gv, out, cyc, reps, busy, active);
    (void)hipDeviceSynchronize();
    long long c;
    (void)hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    printf("%s L=%2d val=%-6s busy=%d active=%2d  %.2f cycles/link\n", bar ? "bar" : "imm", L, VAL == 0 ? "const" : VAL == 1 ? "lds" : "global",
           busy, active, (double)c / ((double)reps * NG * 4));
}

int main()
{
    float *out, *gv;
    long long* cyc;
    (void)hipMalloc(&out, 4096 * 4); (void)hipMalloc(&cyc, 8 * 64); (void)hipMalloc(&gv, W * 4 * 2);
    (void)hipMemset(gv, 0, W * 8);
    run_imm<7, 1>(gv, out, cyc, 0, 32);
    run_imm<7, 1>(gv, out, cyc, 0, 32, true);
    run_imm<7, 0>(gv, out, cyc, 0, 32, true);
    run_imm<4, 1>(gv, out, cyc, 0, 32, true);
    for (int busy : {0})
        for (int active : {32, 64}) {
            run<2, 0>(gv, out, cyc, busy, active);
            run<4, 0>(gv, out, cyc, busy, active);
            run<8, 0>(gv, out, cyc, busy, active);
            run<14, 0>(gv, out, cyc, busy, active);
            run<4, 1>(gv, out, cyc, busy, active);
            run<7, 1>(gv, out, cyc, busy, active);
            run<4, 2>(gv, out, cyc, busy, active);
            run<8, 2>(gv, out, cyc, busy, active);
            run<14, 2>(gv, out, cyc, busy, active);
            run_imm<4, 0>(gv, out, cyc, busy, active);
            run_imm<8, 0>(gv, out, cyc, busy, active);
            run_imm<14, 0>(gv, out, cyc, busy, active);
            run_imm<4, 1>(gv, out, cyc, busy, active);
            run_imm<7, 1>(gv, out, cyc, busy, active);
            run_imm<4, 2>(gv, out, cyc, busy, active);
            run_imm<8, 2>(gv, out, cyc, busy, active);
            run_imm<14, 2>(gv, out, cyc, busy, active);
            run_imm<24, 2>(gv, out, cyc, busy, active);
        }
    return 0;
}
