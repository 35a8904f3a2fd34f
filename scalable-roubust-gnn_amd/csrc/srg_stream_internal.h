// srg_stream_internal.h -- library-internal interface of the LDS-DMA light-row stream (srg_stream.hip),
// used by the hop plan loop in srg_spmm.hip.  Not part of the C-ABI.
#ifndef SRG_STREAM_INTERNAL_H_
#define SRG_STREAM_INTERNAL_H_

#include <hip/hip_runtime.h>

#include <cstdint>

// a row's store and bookkeeping weigh as this many entries when runs are cut (see srg_stream.hip)
constexpr int kStreamRowCost = 4;
// longest run a layout may ask for (its rows' (end, row) pairs sit in the wave's LDS)
constexpr int kStreamMaxWaveEntries = 4096;

// one launch's light rows laid out as a stream (srg_stream_layout_build)
struct SrgStreamRun {
    const int32_t* ent;       // (column id, value bits) pairs; id < 0: the pseudo entry of row -1 - id
    const int64_t* end;       // [n] end position of every row
    const int32_t* row;       // [n] output row
    const int32_t* wave;      // [waves + 1] first row of every wave's run
    int64_t waves;
    int64_t wave_entries;
};

// whether k_stream serves this launch: d in {64, 128, 256}, 16-byte aligned rows
bool srg_stream_fits(const SrgStreamRun& r, const float* X, int64_t ldx, const float* Y, int64_t ldy, int d);
// the light rows' launch (acc: the layout carries a pseudo entry per row, chains start from -0.0f)
int srg_stream_launch(const SrgStreamRun& r, const float* X, int64_t ldx, float* Y, int64_t ldy, int d, int acc,
                      int nt, hipStream_t s);

#endif  // SRG_STREAM_INTERNAL_H_
