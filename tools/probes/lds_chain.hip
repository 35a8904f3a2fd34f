// Microbenchmark: one wave running a dependent fma chain fed by LDS ds_read_b128 (the hub
// consumer's inner loop), alone or next to busy "producer" waves.  Prints cycles per link.
//   hipcc -O3 --offload-arch=gfx950 tools/probes/lds_chain.hip -o /tmp/lds_chain && /tmp/lds_chain
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float V4 __attribute__((ext_vector_type(4)));
constexpr int LD = 528, W = 512;

template <int MODE>   // 0: tile + value reads, 1: tile only, 2: value only, 3: none (registers), 4: tile + DPP-broadcast values
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
            if constexpr (MODE == 4) {
                // sets of 16 links: 4 tile ds_read_b128 + ONE ds_read_b32 of values (lane l holds value
                // l & 15), broadcast per 16-lane row by DPP row_newbcast inside the fma; ring of 3 sets
                struct Set { V4 t[4]; float v; };
                auto ld4 = [&](int set, Set& st) {
                    for (int i = 0; i < 4; ++i)
                        st.t[i] = *reinterpret_cast<const V4*>(tcol + ((((set * 4 + i) & 127) ^ sw) << 2));
                    st.v = av[((set * 16) + (lane & 15)) & 511];
                };
#define F(n, xv) asm volatile("v_fmac_f32_dpp %0, %1, %2 row_newbcast:" #n " row_mask:0xf bank_mask:0xf" : "+v"(acc) : "v"(st.v), "v"(xv))
                auto run4 = [&](const Set& st) {
                    F(0, st.t[0][0]); F(1, st.t[0][1]); F(2, st.t[0][2]); F(3, st.t[0][3]);
                    F(4, st.t[1][0]); F(5, st.t[1][1]); F(6, st.t[1][2]); F(7, st.t[1][3]);
                    F(8, st.t[2][0]); F(9, st.t[2][1]); F(10, st.t[2][2]); F(11, st.t[2][3]);
                    F(12, st.t[3][0]); F(13, st.t[3][1]); F(14, st.t[3][2]); F(15, st.t[3][3]);
                };
#undef F
                Set A, B, C;
                ld4(0, A); __builtin_amdgcn_sched_barrier(0);
                ld4(1, B); __builtin_amdgcn_sched_barrier(0);
                for (int kk = 0; kk + 5 <= 30; kk += 3) {   // 30 sets of 16 = 480 links per rep
                    ld4(kk + 2, C); __builtin_amdgcn_sched_barrier(0);
                    asm volatile("s_waitcnt lgkmcnt(10)" ::: "memory");
                    run4(A); __builtin_amdgcn_sched_barrier(0);
                    ld4(kk + 3, A); __builtin_amdgcn_sched_barrier(0);
                    asm volatile("s_waitcnt lgkmcnt(10)" ::: "memory");
                    run4(B); __builtin_amdgcn_sched_barrier(0);
                    ld4(kk + 4, B); __builtin_amdgcn_sched_barrier(0);
                    asm volatile("s_waitcnt lgkmcnt(10)" ::: "memory");
                    run4(C); __builtin_amdgcn_sched_barrier(0);
                }
                continue;
            }
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
    const char* names[] = {"tile+value", "tile only", "value only", "registers", "tile+dpp"};
    for (int active : {32, 64})
        for (int mode = 0; mode < 5; ++mode) {
            auto fn = mode == 0 ? k<0> : mode == 1 ? k<1> : mode == 2 ? k<2> : mode == 3 ? k<3> : k<4>;
            hipLaunchKernelGGL(fn, dim3(1), dim3(576), 0, 0, in, out, cyc, reps, 0, 0, active);
            (void)hipDeviceSynchronize();
            long long c;
            (void)hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
            const long long l = mode == 4 ? (long long)reps * 9 * 3 * 16 : links;
            printf("active=%2d %-11s %.2f cycles/link\n", active, names[mode], (double)c / l);
        }
    return 0;
}
