// Microbenchmark: cycles per link of one fp32 fma chain (one wave, registers only) when the link's
// value comes by DPP quad broadcast:
//   0: v_fmac_f32 acc, a, x                     (value already in every lane)
//   1: v_fmac_f32_dpp acc, a, x quad_perm       (broadcast fused into the chained fma)
//   2: v_mov_b32_dpp t, a quad_perm; v_fmac_f32 acc, t, x   (broadcast off the chain, in order)
//   3: as 2, with the broadcasts of 4 links issued ahead of their fmas
//   hipcc -O3 --offload-arch=gfx950 tools/probes/dpp_chain.hip -o /tmp/dpp_chain && /tmp/dpp_chain
#include <hip/hip_runtime.h>
#include <cstdio>

#define QP(I) " quad_perm:[" #I "," #I "," #I "," #I "] row_mask:0xf bank_mask:0xf\n"

template <int MODE>
__global__ void k(const float* in, float* out, long long* cyc, int reps)
{
    const int l = threadIdx.x;
    float acc = in[l], a0 = in[l + 64], a1 = in[l + 128], x0 = in[l + 192], x1 = in[l + 256];
    float t0 = 0.f, t1 = 0.f, t2 = 0.f, t3 = 0.f;
    long long c0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < reps; ++r) {
        if (MODE == 0) {
            asm volatile(
                "v_fmac_f32 %0, %1, %3\n v_fmac_f32 %0, %2, %4\n v_fmac_f32 %0, %1, %4\n v_fmac_f32 %0, %2, %3\n"
                "v_fmac_f32 %0, %1, %3\n v_fmac_f32 %0, %2, %4\n v_fmac_f32 %0, %1, %4\n v_fmac_f32 %0, %2, %3\n"
                "v_fmac_f32 %0, %1, %3\n v_fmac_f32 %0, %2, %4\n v_fmac_f32 %0, %1, %4\n v_fmac_f32 %0, %2, %3\n"
                "v_fmac_f32 %0, %1, %3\n v_fmac_f32 %0, %2, %4\n v_fmac_f32 %0, %1, %4\n v_fmac_f32 %0, %2, %3\n"
                : "+v"(acc) : "v"(a0), "v"(a1), "v"(x0), "v"(x1));
        } else if (MODE == 1) {
            asm volatile(
                "v_fmac_f32_dpp %0, %1, %3" QP(0) "v_fmac_f32_dpp %0, %2, %4" QP(0)
                "v_fmac_f32_dpp %0, %1, %4" QP(1) "v_fmac_f32_dpp %0, %2, %3" QP(1)
                "v_fmac_f32_dpp %0, %1, %3" QP(2) "v_fmac_f32_dpp %0, %2, %4" QP(2)
                "v_fmac_f32_dpp %0, %1, %4" QP(3) "v_fmac_f32_dpp %0, %2, %3" QP(3)
                "v_fmac_f32_dpp %0, %1, %3" QP(0) "v_fmac_f32_dpp %0, %2, %4" QP(0)
                "v_fmac_f32_dpp %0, %1, %4" QP(1) "v_fmac_f32_dpp %0, %2, %3" QP(1)
                "v_fmac_f32_dpp %0, %1, %3" QP(2) "v_fmac_f32_dpp %0, %2, %4" QP(2)
                "v_fmac_f32_dpp %0, %1, %4" QP(3) "v_fmac_f32_dpp %0, %2, %3" QP(3)
                : "+v"(acc) : "v"(a0), "v"(a1), "v"(x0), "v"(x1));
        } else if (MODE == 2) {
            asm volatile(
                "v_mov_b32_dpp %1, %5" QP(0) "v_fmac_f32 %0, %1, %7\n"
                "v_mov_b32_dpp %2, %6" QP(0) "v_fmac_f32 %0, %2, %8\n"
                "v_mov_b32_dpp %3, %5" QP(1) "v_fmac_f32 %0, %3, %8\n"
                "v_mov_b32_dpp %4, %6" QP(1) "v_fmac_f32 %0, %4, %7\n"
                "v_mov_b32_dpp %1, %5" QP(2) "v_fmac_f32 %0, %1, %7\n"
                "v_mov_b32_dpp %2, %6" QP(2) "v_fmac_f32 %0, %2, %8\n"
                "v_mov_b32_dpp %3, %5" QP(3) "v_fmac_f32 %0, %3, %8\n"
                "v_mov_b32_dpp %4, %6" QP(3) "v_fmac_f32 %0, %4, %7\n"
                "v_mov_b32_dpp %1, %5" QP(0) "v_fmac_f32 %0, %1, %7\n"
                "v_mov_b32_dpp %2, %6" QP(0) "v_fmac_f32 %0, %2, %8\n"
                "v_mov_b32_dpp %3, %5" QP(1) "v_fmac_f32 %0, %3, %8\n"
                "v_mov_b32_dpp %4, %6" QP(1) "v_fmac_f32 %0, %4, %7\n"
                "v_mov_b32_dpp %1, %5" QP(2) "v_fmac_f32 %0, %1, %7\n"
                "v_mov_b32_dpp %2, %6" QP(2) "v_fmac_f32 %0, %2, %8\n"
                "v_mov_b32_dpp %3, %5" QP(3) "v_fmac_f32 %0, %3, %8\n"
                "v_mov_b32_dpp %4, %6" QP(3) "v_fmac_f32 %0, %4, %7\n"
                : "+v"(acc), "+v"(t0), "+v"(t1), "+v"(t2), "+v"(t3) : "v"(a0), "v"(a1), "v"(x0), "v"(x1));
        } else {
            asm volatile(
                "v_mov_b32_dpp %1, %5" QP(0) "v_mov_b32_dpp %2, %6" QP(0)
                "v_mov_b32_dpp %3, %5" QP(1) "v_mov_b32_dpp %4, %6" QP(1)
                "v_fmac_f32 %0, %1, %7\n v_fmac_f32 %0, %2, %8\n v_fmac_f32 %0, %3, %8\n v_fmac_f32 %0, %4, %7\n"
                "v_mov_b32_dpp %1, %5" QP(2) "v_mov_b32_dpp %2, %6" QP(2)
                "v_mov_b32_dpp %3, %5" QP(3) "v_mov_b32_dpp %4, %6" QP(3)
                "v_fmac_f32 %0, %1, %7\n v_fmac_f32 %0, %2, %8\n v_fmac_f32 %0, %3, %8\n v_fmac_f32 %0, %4, %7\n"
                "v_mov_b32_dpp %1, %5" QP(0) "v_mov_b32_dpp %2, %6" QP(0)
                "v_mov_b32_dpp %3, %5" QP(1) "v_mov_b32_dpp %4, %6" QP(1)
                "v_fmac_f32 %0, %1, %7\n v_fmac_f32 %0, %2, %8\n v_fmac_f32 %0, %3, %8\n v_fmac_f32 %0, %4, %7\n"
                "v_mov_b32_dpp %1, %5" QP(2) "v_mov_b32_dpp %2, %6" QP(2)
                "v_mov_b32_dpp %3, %5" QP(3) "v_mov_b32_dpp %4, %6" QP(3)
                "v_fmac_f32 %0, %1, %7\n v_fmac_f32 %0, %2, %8\n v_fmac_f32 %0, %3, %8\n v_fmac_f32 %0, %4, %7\n"
                : "+v"(acc), "+v"(t0), "+v"(t1), "+v"(t2), "+v"(t3) : "v"(a0), "v"(a1), "v"(x0), "v"(x1));
        }
    }
    long long c1 = __builtin_amdgcn_s_memtime();
    out[l] = acc + t0 + t1 + t2 + t3;
    if (l == 0) cyc[0] = c1 - c0;
}

int main()
{
    float *in, *out;
    long long* cyc;
    hipMalloc(&in, 320 * 4);
    hipMalloc(&out, 64 * 4);
    hipMalloc(&cyc, 8);
    hipMemset(in, 0, 320 * 4);
    const int reps = 20000;
    const char* names[] = {"fmac (value in every lane)", "fmac_dpp (broadcast fused)", "mov_dpp + fmac, in order",
                           "mov_dpp x4 ahead + fmac x4"};
    for (int m = 0; m < 4; ++m) {
        for (int it = 0; it < 2; ++it) {
            if (m == 0) hipLaunchKernelGGL(k<0>, dim3(1), dim3(64), 0, 0, in, out, cyc, reps);
            if (m == 1) hipLaunchKernelGGL(k<1>, dim3(1), dim3(64), 0, 0, in, out, cyc, reps);
            if (m == 2) hipLaunchKernelGGL(k<2>, dim3(1), dim3(64), 0, 0, in, out, cyc, reps);
            if (m == 3) hipLaunchKernelGGL(k<3>, dim3(1), dim3(64), 0, 0, in, out, cyc, reps);
            hipDeviceSynchronize();
        }
        long long c;
        hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
        // s_memtime counts at the shader clock
        printf("%-30s %6.2f cycles/link\n", names[m], (double)c / (reps * 16.0));
    }
    return 0;
}
