// Microbenchmark: one wave running a dependent fma chain fed by LDS ds_read_b128 (the hub
// consumer's inner loop), alone or next to busy "producer" waves.  Prints cycles per link.
//   hipcc -O3 --offload-arch=gfx950 tools/probes/lds_chain.hip -o /tmp/lds_chain && /tmp/lds_chain
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float V4 __attribute__((ext_vector_type(4)));
constexpr int LD = 528, W = 512;

template <int MODE>   // 0: tile + value reads, 1: tile only, 2: value only, 3: none (registers)
__global__ void __launch_bounds__(576) k(const float* in, float* out, long long* cyc, int reps, int busy, int prio, int active)
{
    __shared__ __attribute__((aligned(16))) float lds[32 * LD + W];
    for (int i = threadIdx.x; i < 32 * LD + W; i += blockDim.x) lds[i] = in[i];
    __syncthreads();
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (wave != 0) {   // producers: optionally burn VALU / LDS writes
        float x = lane;
        if (busy == 1) for (int r = 0; r < reps * 64; ++r) x = __builtin_fmaf(x, 0.999f, 0.5f);
        if (busy == 2) for (int r = 0; r < reps * 16; ++r) lds[(lane * 33 + r) % (32 * LD)] = x;
        if (x == 12345.f) out[1] = x;
        return;
    }
    if (prio) __builtin_amdgcn_s_setprio(3);
    const int c = lane & 31, sw = (c >> 2) & 7;
    const float* tcol = lds + c * LD;
    const float* av = lds + 32 * LD;
    float acc = 0.f;
    long long t0 = clock64();
    if (lane < active) {
        for (int r = 0; r < reps; ++r) {
            asm volatile("" ::: "memory");
            V4 t[4][2], a[4][2];
            auto ld = [&](int set, V4 (&tt)[2], V4 (&aa)[2]) {
                for (int i = 0; i < 2; ++i) {
                    int grp = (set * 2 + i) & 127;
                    if (MODE == 0 || MODE == 1) tt[i] = *reinterpret_cast<const V4*>(tcol + ((grp ^ sw) << 2));
                    else tt[i] = V4{1.f, 1.f, 1.f, 1.f};
                    if (MODE == 0 || MODE == 2) aa[i] = *reinterpret_cast<const V4*>(av + (grp << 2));
                    else aa[i] = V4{0.5f, 0.5f, 0.5f, 0.5f};
                }
            };
            auto run = [&](const V4 (&tt)[2], const V4 (&aa)[2]) {
                for (int i = 0; i < 2; ++i)
                    for (int e = 0; e < 4; ++e) acc = __builtin_fmaf(aa[i][e], tt[i][e], acc);
            };
            ld(0, t[0], a[0]); __builtin_amdgcn_sched_barrier(0);
            ld(1, t[1], a[1]); __builtin_amdgcn_sched_barrier(0);
            ld(2, t[2], a[2]); __builtin_amdgcn_sched_barrier(0);
            for (int kk = 0; kk + 7 <= 64; kk += 4) {
                ld(kk + 3, t[3], a[3]); __builtin_amdgcn_sched_barrier(0);
                run(t[0], a[0]); __builtin_amdgcn_sched_barrier(0);
                ld(kk + 4, t[0], a[0]); __builtin_amdgcn_sched_barrier(0);
                run(t[1], a[1]); __builtin_amdgcn_sched_barrier(0);
                ld(kk + 5, t[1], a[1]); __builtin_amdgcn_sched_barrier(0);
                run(t[2], a[2]); __builtin_amdgcn_sched_barrier(0);
                ld(kk + 6, t[2], a[2]); __builtin_amdgcn_sched_barrier(0);
                run(t[3], a[3]); __builtin_amdgcn_sched_barrier(0);
            }
        }
    }
    long long t1 = clock64();
    if (lane == 0) cyc[blockIdx.x] = t1 - t0;
    out[threadIdx.x] = acc;
}

int main()
{
    float* out; long long* cyc; float* in;
    (void)hipMalloc(&out, 4096 * 4); (void)hipMalloc(&cyc, 8 * 1024); (void)hipMalloc(&in, (32 * LD + W) * 4);
    (void)hipMemset(in, 0, (32 * LD + W) * 4);
    const int reps = 200;
    const long long links = (long long)reps * 15 * 4 * 8;   // 15 iterations x 4 sets x 8 links
    const char* names[] = {"tile+value", "tile only", "value only", "registers"};
    for (int active : {4, 8, 16, 32, 64})
        for (int mode = 0; mode < 4; ++mode) {
            auto fn = mode == 0 ? k<0> : mode == 1 ? k<1> : mode == 2 ? k<2> : k<3>;
            hipLaunchKernelGGL(fn, dim3(1), dim3(576), 0, 0, in, out, cyc, reps, 0, 0, active);
            (void)hipDeviceSynchronize();
            long long c;
            (void)hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
            printf("active=%2d %-11s %.2f cycles/link\n", active, names[mode], (double)c / links);
        }
    return 0;
}
