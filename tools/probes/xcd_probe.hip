// Probe (not product code): does giving each XCD its own column block raise the L2 share enough to
// pay?  B = 8 column blocks of the products hop (every row cut), each a compact CSR with its own
// schedule and its own output panel (results are NOT combined: a throughput probe).  One persistent
// kernel runs the library's own slice-wave / packed-row device code over work items taken from a
// per-block counter:
//   mode 0: a workgroup works on block XCC_ID (its XCD's block): each XCD's L2 caches one slice of X;
//   mode 1: every workgroup works on block `fixed` (one launch per block, the sequential B = 8 hop);
//   mode 2: a workgroup works on block (blockIdx / 8) % 8: all blocks at once on every XCD (control).
// Hub rows are left out (the schedule passed starts after them).
//   hipcc -O3 -std=c++17 -fPIC -shared --offload-arch=gfx950 -ffp-contract=off -Iinclude \
//       tools/probes/xcd_probe.hip -o tools/probes/_build/libxcd_probe.so
#include "../../scalable-roubust-gnn_amd/csrc/srg_spmm.hip"

namespace {

struct XBlk {   // all int64 (filled from a host int64 array)
    int64_t indptr, indices, vals, order, Y, n_rows, n_heavy, nb_heavy, n_blocks;
};

__device__ __forceinline__ int xcc_id()
{
    int v;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(v));
    return v;
}

template <int LR, int LQ, int U>
__global__ void __launch_bounds__(kBlock)
k_xprobe(const XBlk* __restrict__ blks, int mode, int fixed, int* __restrict__ ctr, int* __restrict__ xlog,
         int n_slices, const float* __restrict__ X, int64_t ldx, int d)
{
    __shared__ __attribute__((aligned(16))) float lds[kWavesPerBlock * 256];
    __shared__ int s_bid;
    const int wib = threadIdx.x >> 6;
    const int b = mode == 0 ? (xcc_id() & 7) : mode == 1 ? fixed : (int)((blockIdx.x >> 3) & 7);
    if (xlog && threadIdx.x == 0) xlog[blockIdx.x] = xcc_id();
    const XBlk B = blks[b];
    const int64_t* ip = reinterpret_cast<const int64_t*>(B.indptr);
    const int32_t* ix = reinterpret_cast<const int32_t*>(B.indices);
    const float* vv = reinterpret_cast<const float*>(B.vals);
    const int32_t* order = reinterpret_cast<const int32_t*>(B.order);
    float* Y = reinterpret_cast<float*>(B.Y);
    const int n_rows = (int)B.n_rows, n_heavy = (int)B.n_heavy, nb_heavy = (int)B.nb_heavy;
    const int n_blocks = (int)B.n_blocks;
    Epi epi{};
    for (;;) {
        if (threadIdx.x == 0) s_bid = atomicAdd(&ctr[b], 1);
        __syncthreads();
        const int bid = s_bid;
        __syncthreads();
        if (bid >= n_blocks) break;            // workgroup-uniform: every wave leaves together
        if (bid < nb_heavy) {
            const int item = __builtin_amdgcn_readfirstlane(bid * kWavesPerBlock + wib);
            if (item < n_heavy * n_slices)
                slice_wave<kUnrollHeavy, true, int64_t, kEpiPlain>(ip, ix, vv, order[item / n_slices], item % n_slices,
                                                                   X, ldx, Y, ldx, d, 0, 0, lds + wib * 256, epi);
        } else {
            const int first = __builtin_amdgcn_readfirstlane((bid - nb_heavy) * kWavesPerBlock + wib) * LR + n_heavy;
            if (first < n_rows)
                packed_rows<LR, LQ, U, int64_t, kEpiPlain>(ip, ix, vv, order, n_rows, first, X, ldx, Y, ldx, 0, 0, epi);
        }
    }
}

}  // namespace

extern "C" int xprobe_run(const void* blks, int mode, int fixed, int* ctr, int* xlog, int grid, int n_slices,
                          const float* X, int64_t ldx, int d, void* stream)
{
    if (d != 128 || ldx % 4) return fail(SRG_ERR_INVALID, "probe is for d = 128");
    hipLaunchKernelGGL((k_xprobe<4, 2, 2>), dim3(grid), dim3(kBlock), 0, (hipStream_t)stream,
                       (const XBlk*)blks, mode, fixed, ctr, xlog, n_slices, X, ldx, d);
    SRG_HIP_CHECK(hipGetLastError());
    return SRG_OK;
}
