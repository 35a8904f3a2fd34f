// srg_halo_internal.h -- library-internal layout of the halo-exchange plan and device share shared by
// srg_halo.hip (the host planner, the share's device arrays) and srg_comm.hip (the per-hop executor
// over RCCL or the loopback transport).  Not part of the C-ABI: include/srgnn_hip.h holds the opaque
// handles.
#ifndef SRG_HALO_INTERNAL_H_
#define SRG_HALO_INTERNAL_H_

#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

#include "srgnn_hip.h"

// one launch of the hop: a row schedule over the local CSR (a row chunk, the hub group, the ghosts)
struct SrgHaloView {
    std::vector<int32_t> order;    // local row ids (panel rows), longest first
    int64_t n = 0;                 // rows scheduled
    int64_t n_hub = 0;             // hub workgroup rows (the hub group: all of them)
    int64_t n_heavy = 0;           // slice-wave rows for d > 32
    int64_t n_heavy_narrow = 0;    // slice-wave rows for d <= 32
};

// rank p's share of the halo-exchange partition (srgnn/dist.py HaloPartitionedOperator, restated in
// C++ for C hosts): everything is derived from the global CSR, identically on every rank
struct srg_halo_plan {
    int32_t P = 1, p = 0, C = 1;                  // ranks, this rank, row chunks (groups C + 1: + hub group)
    int64_t n = 0, nnz_total = 0;
    int64_t r0 = 0, r1 = 0, rows = 0;             // own rows [r0, r1)
    int64_t b0 = 0, b1 = 0;                        // own entries [b0, b1) of the global CSR
    int64_t n_recv = 0, n_ghost = 0, halo = 0;
    int32_t ghost_max_degree = 0;
    int64_t heavy_threshold = 0;                   // the chunks' slice-wave threshold used
    bool auto_heavy = true;                        // heavy_threshold was SRG_HALO_AUTO
    std::vector<int64_t> hub_thresholds;           // per owner rank
    std::vector<int64_t> starts;                   // [P + 1] row blocks
    std::vector<int64_t> chunk_ranges;             // [C + 1] local row bounds of this rank's chunks
    // local CSR over the panel rows [own | received (empty) | ghosts], columns remapped into the panel
    std::vector<int64_t> lip;                      // [rows + halo + 1]
    std::vector<int32_t> lix;
    std::vector<int64_t> ghost_pos;                // global entry positions of the ghost rows' entries
    std::vector<SrgHaloView> views;                // C chunks, the hub group, the ghost rows
    // exchange: group g = chunk g (g < C) or the hub group (g == C)
    std::vector<std::vector<int64_t>> recv_counts; // [G][P] rows received per (group, source)
    std::vector<int64_t> group_offsets;            // [G] start of a group's rows inside the halo
    std::vector<std::vector<int64_t>> send_counts; // [G][P]
    std::vector<std::vector<int64_t>> send_cat;    // [G] local row ids sent, peers ascending
    std::vector<int64_t> ghost_recv_counts, ghost_send_counts;   // [P] (the first exchange of X only)
    std::vector<int64_t> ghost_send_cat;
    std::vector<int64_t> halo_ids;                 // global ids of the halo rows, panel order
};

// The row chunks' column blocks (srgnn/dist.py HaloPartitionedOperator.chunk_blocks): block b of an own
// row is its span [bounds[b][r], bounds[b+1][r]) of the local CSR, cut where the entries' GLOBAL column
// ids cross ceil(b n / B); rows of <= BLOCK_WHOLE_MAX (48) entries run whole in block 0.  Chunk c's block 0
// schedules all its rows, blocks 1.. its cut rows; each launch continues the chains of the one before
// (ACCUMULATE), so every row is the unblocked fma chain.
struct SrgHaloBlocks {
    int B = 1;                                     // 1: the chunks run unblocked
    bool forced = false;                           // set by srg_halo_share_col_blocks: for every d
    std::vector<const int64_t*> bounds;            // [B + 1] device: lip, the B - 1 split arrays, lip + 1
    std::vector<int64_t*> splits;                  // the B - 1 allocated split arrays [rows]
    std::vector<std::vector<SrgHaloView>> views;   // [C][B]: rows, heavy counts (order kept on the host only while built)
    std::vector<std::vector<int32_t*>> orders;     // [C][B] device schedules
};

// column blocks per row-chunk launch for a d-column panel of `nloc` rows (dist.py _col_blocks_for):
// 8 for panels >= 8 GiB at d >= 256, else 1 (srg_halo_share_col_blocks sets a count for every d)
int srg_halo_col_blocks(int64_t nloc, int d);

struct srg_halo_share {
    int device = 0;
    const srg_halo_plan* plan = nullptr;           // borrowed: must outlive the share
    int64_t* lip = nullptr;
    int32_t* lix = nullptr;
    float* lvv = nullptr;
    SrgHaloBlocks blocks;                          // for d_max's block count
    std::vector<int32_t*> orders;                  // per view (device)
    std::vector<int64_t*> send_idx;                // per group (device), then the ghost sends
    std::vector<int64_t> send_off;                 // [G + 2] rows of the send buffer per group, ghosts last
    float* sendbuf = nullptr;                      // [send_off.back(), d_cap]
    int64_t d_cap = 0;
    std::vector<hipEvent_t> packed;                // per group + ghosts: the pack is on the shard's stream
    hipStream_t comm_stream = nullptr;             // RCCL's stream of this shard
    hipEvent_t comm_done = nullptr;
    bool counts_verified = false;                  // its peers agreed on every exchange count (first RCCL call)
};

#endif  // SRG_HALO_INTERNAL_H_
