// srg_comm.hip -- communicator lifecycle and the row-partitioned K-hop propagation over RCCL, for C / C++
// hosts (the Python package drives the same kernels through torch.distributed,
// srgnn/dist.py).
//
// Partition: rank r owns rows [row_starts[r], row_starts[r+1]) of Â (a 1-D, contiguous row block with
// global column ids) and the same rows of every hop panel.  srg_dist_propagate_khop_f32 is SURVEY §8(e)'s
// all-gather, chunked by owner and overlapped with the SpMM: per hop every pair of ranks exchanges its
// blocks of the previous panel in a grouped ncclSend / ncclRecv on a stream of that pair (all links at
// once), and each rank multiplies its rows in P column blocks -- block q = the entries whose column ids
// lie in rank q's rows, a span of every row since Â's rows hold sorted ids -- in ascending q, block q
// as soon as rank q's rows have arrived (the own block first copied locally), blocks 1.. continuing
// the chains of block 0 (SRG_SPMM_ACCUMULATE).  Every row's fma chain is the one-GPU chain in CSR order,
// so every hop is bitwise the one-GPU hop.  The halo exchange (srg_halo_*, below) moves only the rows
// each rank references and is the faster path.
//
// RCCL is loaded at run time (dlopen, RTLD_LOCAL): a process that already holds an RCCL (PyTorch's) keeps
// using that one, and the library itself has no link-time dependency on it.  SRGNN_RCCL_LIB names a
// specific librccl (the tests load an in-process stand-in, tests/fake_rccl.cpp, to run these RCCL paths
// with several ranks on one GPU).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <dlfcn.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <vector>

#include "srg_halo_internal.h"
#include "srgnn_hip.h"

extern "C" void srg_set_error(int code, const char* msg);   // srg_spmm.hip: thread-local srg_last_error

namespace {

int comm_fail(int code, const char* fmt, ...)
{
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    srg_set_error(code, buf);
    return code;
}

struct Rccl {
    void* handle = nullptr;
    ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
    ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*CommInitAll)(ncclComm_t*, int, const int*) = nullptr;
    ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*GroupStart)() = nullptr;
    ncclResult_t (*GroupEnd)() = nullptr;
    ncclResult_t (*Send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*Recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    const char* (*GetErrorString)(ncclResult_t) = nullptr;
};

std::mutex g_rccl_mu;
Rccl g_rccl;

template <typename F>
bool sym(void* h, const char* name, F& out)
{
    out = reinterpret_cast<F>(dlsym(h, name));
    return out != nullptr;
}

int load_rccl(const Rccl** out)
{
    std::lock_guard<std::mutex> lock(g_rccl_mu);
    if (!g_rccl.handle) {
        void* h = nullptr;
        const char* env = getenv("SRGNN_RCCL_LIB");
        if (env && *env) {
            h = dlopen(env, RTLD_NOW | RTLD_LOCAL);
        } else {
            // an RCCL this process already loaded (PyTorch's) first, then the system one
            const char* names[] = {"librccl.so", "librccl.so.1"};
            for (const char* n : names)
                if (!h) h = dlopen(n, RTLD_NOW | RTLD_NOLOAD);
            for (const char* n : names)
                if (!h) h = dlopen(n, RTLD_NOW | RTLD_LOCAL);
            if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        }
        if (!h) return comm_fail(SRG_ERR_HIP, "cannot load librccl: %s", dlerror());
        Rccl r;
        r.handle = h;
        if (!sym(h, "ncclGetUniqueId", r.GetUniqueId) || !sym(h, "ncclCommInitRank", r.CommInitRank) ||
            !sym(h, "ncclCommInitAll", r.CommInitAll) || !sym(h, "ncclCommDestroy", r.CommDestroy) ||
            !sym(h, "ncclGroupStart", r.GroupStart) || !sym(h, "ncclGroupEnd", r.GroupEnd) ||
            !sym(h, "ncclSend", r.Send) || !sym(h, "ncclRecv", r.Recv) ||
            !sym(h, "ncclGetErrorString", r.GetErrorString))
            return comm_fail(SRG_ERR_HIP, "librccl lacks an entry point: %s", dlerror());
        g_rccl = r;
    }
    *out = &g_rccl;
    return SRG_OK;
}

#define SRG_NCCL(r, expr)                                                                        \
    do {                                                                                         \
        ncclResult_t e_ = (expr);                                                                \
        if (e_ != ncclSuccess)                                                                   \
            return comm_fail(SRG_ERR_HIP, "%s failed: %s", #expr, (r)->GetErrorString(e_));      \
    } while (0)

#define SRG_HIPC(expr)                                                                           \
    do {                                                                                         \
        hipError_t e_ = (expr);                                                                  \
        if (e_ != hipSuccess)                                                                    \
            return comm_fail(SRG_ERR_HIP, "%s failed: %s", #expr, hipGetErrorString(e_));        \
    } while (0)

struct DeviceScope {   // current device restored on exit
    int prev = -1;
    DeviceScope() { if (hipGetDevice(&prev) != hipSuccess) prev = -1; }
    ~DeviceScope() { if (prev >= 0) (void)hipSetDevice(prev); }
};

}  // namespace

struct srg_comm {
    int nranks = 0;
    std::vector<ncclComm_t> comms;   // one per local device
    std::vector<int> ranks;          // their global ranks
    std::vector<int> devices;
    // loopback: every rank in this process on one device, exchanges by device copies (no RCCL)
    bool loopback = false;
    hipStream_t lb_stream = nullptr;
    hipEvent_t lb_done = nullptr;
    // srg_dist_propagate_khop_f32: per local rank, a stream and an arrival event per peer, and the
    // "previous panel ready" event (created on first use)
    std::vector<std::vector<hipStream_t>> peer_stream;
    std::vector<std::vector<hipEvent_t>> peer_arrived;
    std::vector<hipEvent_t> panel_ready;
};

namespace {

// splits[(b - 1) * n + r] = the first entry of row r whose column id is >= bounds[b], b = 1 .. P - 1 (one
// wave per row: a binary search per boundary, and a check that the row's ids never decrease -- else
// a block would read rows of another owner before they arrive)
__global__ void __launch_bounds__(256)
k_owner_splits(const int64_t* __restrict__ indptr, const int32_t* __restrict__ indices, int64_t n,
               const int64_t* __restrict__ bounds, int P, int64_t* __restrict__ splits, int* __restrict__ bad)
{
    const int lane = threadIdx.x & 63;
    const int64_t waves = (int64_t)gridDim.x * (blockDim.x / 64);
    for (int64_t r = (int64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6); r < n; r += waves) {
        const int64_t b0 = indptr[r], b1 = indptr[r + 1];
        int unsorted = 0;
        for (int64_t e = b0 + lane; e + 1 < b1; e += 64) unsorted |= indices[e] > indices[e + 1];
        if (__any(unsorted) && lane == 0) atomicOr(bad, 1);
        for (int b = 1 + lane; b < P; b += 64) {
            int64_t lo = b0, hi = b1;
            while (lo < hi) {
                const int64_t mid = lo + (hi - lo) / 2;
                if ((int64_t)indices[mid] < bounds[b])
                    lo = mid + 1;
                else
                    hi = mid;
            }
            splits[(int64_t)(b - 1) * n + r] = lo;
        }
    }
}

// the pair streams and events of srg_dist_propagate_khop_f32 (created once per communicator)
int dist_streams(srg_comm* comm)
{
    const size_t L = comm->comms.size();
    if (comm->peer_stream.size() == L) return SRG_OK;
    comm->peer_stream.assign(L, std::vector<hipStream_t>(comm->nranks, nullptr));
    comm->peer_arrived.assign(L, std::vector<hipEvent_t>(comm->nranks, nullptr));
    comm->panel_ready.assign(L, nullptr);
    for (size_t i = 0; i < L; ++i) {
        SRG_HIPC(hipSetDevice(comm->devices[i]));
        SRG_HIPC(hipEventCreateWithFlags(&comm->panel_ready[i], hipEventDisableTiming));
        for (int q = 0; q < comm->nranks; ++q) {
            if (q == comm->ranks[i]) continue;
            SRG_HIPC(hipStreamCreateWithFlags(&comm->peer_stream[i][q], hipStreamNonBlocking));
            SRG_HIPC(hipEventCreateWithFlags(&comm->peer_arrived[i][q], hipEventDisableTiming));
        }
    }
    return SRG_OK;
}

// One hop's exchange: for every pair of ranks (a, b), a < b, in ascending order, one group with the
// local ranks' send of their block to the other and receive of the other's block into x_full, on the
// pair's stream (which first waits for the previous panel), then the arrival event.  A rank meets its
// peers in ascending order, so the blocks it needs first are sent first; the pairs' streams run
// side by side (every xGMI link at once).
int dist_exchange(const Rccl* r, srg_comm* comm, const srg_shard_f32* shards, int n_shards, const int64_t* row_starts,
                  int64_t ld, int k)
{
    const int P = comm->nranks;
    for (int a = 0; a < P; ++a)
        for (int b = a + 1; b < P; ++b) {
            int local[2] = {-1, -1};
            for (int i = 0; i < n_shards; ++i) {
                if (comm->ranks[i] == a) local[0] = i;
                if (comm->ranks[i] == b) local[1] = i;
            }
            if (local[0] < 0 && local[1] < 0) continue;
            for (int side = 0; side < 2; ++side) {
                const int i = local[side];
                if (i < 0) continue;
                const int peer = side ? a : b;
                SRG_HIPC(hipSetDevice(shards[i].device));
                SRG_HIPC(hipStreamWaitEvent(comm->peer_stream[i][peer], comm->panel_ready[i], 0));
            }
            SRG_NCCL(r, r->GroupStart());
            int rc = SRG_OK;
            for (int side = 0; side < 2 && !rc; ++side) {
                const int i = local[side];
                if (i < 0) continue;
                const srg_shard_f32& s = shards[i];
                const int peer = side ? a : b;
                const hipStream_t ps = comm->peer_stream[i][peer];
                const size_t n_me = (size_t)s.n_rows * (size_t)ld;
                const size_t n_peer = (size_t)(row_starts[peer + 1] - row_starts[peer]) * (size_t)ld;
                ncclResult_t e = ncclSuccess;
                // the previous panel's own rows (complete at panel_ready)
                if (n_me) e = r->Send(s.panels[k - 1], n_me, ncclFloat32, peer, comm->comms[i], ps);
                if (e == ncclSuccess && n_peer)
                    e = r->Recv(s.x_full + (size_t)row_starts[peer] * ld, n_peer, ncclFloat32, peer, comm->comms[i], ps);
                if (e != ncclSuccess) rc = comm_fail(SRG_ERR_HIP, "ncclSend / ncclRecv failed: %s", r->GetErrorString(e));
            }
            // every exit closes the group (RCCL's group state is thread-local and shared with torch)
            const ncclResult_t ge = r->GroupEnd();
            if (rc) return rc;
            if (ge != ncclSuccess) return comm_fail(SRG_ERR_HIP, "ncclGroupEnd failed: %s", r->GetErrorString(ge));
            for (int side = 0; side < 2; ++side) {
                const int i = local[side];
                if (i < 0) continue;
                const int peer = side ? a : b;
                SRG_HIPC(hipSetDevice(shards[i].device));
                SRG_HIPC(hipEventRecord(comm->peer_arrived[i][peer], comm->peer_stream[i][peer]));
            }
        }
    return SRG_OK;
}

}  // namespace

extern "C" {

int srg_comm_unique_id(void* id_out)
{
    if (!id_out) return comm_fail(SRG_ERR_INVALID, "null id buffer");
    const Rccl* r = nullptr;
    int rc = load_rccl(&r);
    if (rc) return rc;
    ncclUniqueId id;
    SRG_NCCL(r, r->GetUniqueId(&id));
    memcpy(id_out, &id, sizeof(id));
    return SRG_OK;
}

int srg_comm_init_rank(int nranks, const void* id, int rank, int device, srg_comm** out)
{
    if (!out || !id) return comm_fail(SRG_ERR_INVALID, "null argument");
    *out = nullptr;
    if (nranks < 1 || rank < 0 || rank >= nranks) return comm_fail(SRG_ERR_INVALID, "rank %d of %d", rank, nranks);
    const Rccl* r = nullptr;
    int rc = load_rccl(&r);
    if (rc) return rc;
    DeviceScope scope;
    SRG_HIPC(hipSetDevice(device));
    ncclUniqueId uid;
    memcpy(&uid, id, sizeof(uid));
    ncclComm_t c = nullptr;
    SRG_NCCL(r, r->CommInitRank(&c, nranks, uid, rank));
    srg_comm* comm = new (std::nothrow) srg_comm();
    if (!comm) {
        (void)r->CommDestroy(c);
        return comm_fail(SRG_ERR_ALLOC, "out of host memory");
    }
    comm->nranks = nranks;
    comm->comms = {c};
    comm->ranks = {rank};
    comm->devices = {device};
    *out = comm;
    return SRG_OK;
}

int srg_comm_init_all(int ndev, const int* devices, srg_comm** out)
{
    if (!out) return comm_fail(SRG_ERR_INVALID, "null argument");
    *out = nullptr;
    if (ndev < 1) return comm_fail(SRG_ERR_INVALID, "ndev=%d < 1", ndev);
    const Rccl* r = nullptr;
    int rc = load_rccl(&r);
    if (rc) return rc;
    std::vector<int> devs(ndev);
    for (int i = 0; i < ndev; ++i) devs[i] = devices ? devices[i] : i;
    std::vector<ncclComm_t> cs(ndev, nullptr);
    DeviceScope scope;
    SRG_NCCL(r, r->CommInitAll(cs.data(), ndev, devs.data()));
    srg_comm* comm = new (std::nothrow) srg_comm();
    if (!comm) {
        for (auto c : cs) (void)r->CommDestroy(c);
        return comm_fail(SRG_ERR_ALLOC, "out of host memory");
    }
    comm->nranks = ndev;
    comm->comms = cs;
    comm->devices = devs;
    for (int i = 0; i < ndev; ++i) comm->ranks.push_back(i);
    *out = comm;
    return SRG_OK;
}

int srg_comm_init_loopback(int nranks, int device, srg_comm** out)
{
    if (!out) return comm_fail(SRG_ERR_INVALID, "null argument");
    *out = nullptr;
    if (nranks < 1) return comm_fail(SRG_ERR_INVALID, "nranks=%d < 1", nranks);
    DeviceScope scope;
    SRG_HIPC(hipSetDevice(device));
    srg_comm* comm = new (std::nothrow) srg_comm();
    if (!comm) return comm_fail(SRG_ERR_ALLOC, "out of host memory");
    comm->nranks = nranks;
    comm->loopback = true;
    for (int i = 0; i < nranks; ++i) {
        comm->ranks.push_back(i);
        comm->devices.push_back(device);
    }
    if (hipStreamCreateWithFlags(&comm->lb_stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&comm->lb_done, hipEventDisableTiming) != hipSuccess) {
        srg_comm_destroy(comm);
        return comm_fail(SRG_ERR_HIP, "loopback stream / event creation failed");
    }
    *out = comm;
    return SRG_OK;
}

int srg_comm_destroy(srg_comm* comm)
{
    if (!comm) return SRG_OK;
    if (comm->loopback) {
        DeviceScope scope;
        (void)hipSetDevice(comm->devices.empty() ? 0 : comm->devices[0]);
        if (comm->lb_stream) {
            (void)hipStreamSynchronize(comm->lb_stream);
            (void)hipStreamDestroy(comm->lb_stream);
        }
        if (comm->lb_done) (void)hipEventDestroy(comm->lb_done);
        delete comm;
        return SRG_OK;
    }
    {
        DeviceScope scope;
        for (size_t i = 0; i < comm->peer_stream.size(); ++i) {
            (void)hipSetDevice(comm->devices[i]);
            for (auto st : comm->peer_stream[i])
                if (st) {
                    (void)hipStreamSynchronize(st);
                    (void)hipStreamDestroy(st);
                }
            for (auto ev : comm->peer_arrived[i])
                if (ev) (void)hipEventDestroy(ev);
            if (comm->panel_ready[i]) (void)hipEventDestroy(comm->panel_ready[i]);
        }
    }
    const Rccl* r = nullptr;
    int rc = load_rccl(&r);
    if (rc) return rc;
    int first = SRG_OK;
    for (auto c : comm->comms) {
        ncclResult_t e = r->CommDestroy(c);
        if (e != ncclSuccess && first == SRG_OK)
            first = comm_fail(SRG_ERR_HIP, "ncclCommDestroy failed: %s", r->GetErrorString(e));
    }
    delete comm;
    return first;
}

int srg_comm_size(const srg_comm* comm) { return comm ? comm->nranks : 0; }

int srg_dist_propagate_khop_f32(srg_comm* comm, const srg_shard_f32* shards, int n_shards,
                                const int64_t* row_starts, int64_t ld, int32_t d, int32_t K)
{
    if (!comm || !shards || !row_starts) return comm_fail(SRG_ERR_INVALID, "null argument");
    if (comm->loopback) return comm_fail(SRG_ERR_INVALID, "a loopback communicator serves srg_halo_propagate_f32 only");
    if (n_shards != (int)comm->comms.size())
        return comm_fail(SRG_ERR_INVALID, "%d shards for %d local ranks", n_shards, (int)comm->comms.size());
    if (K < 0 || d < 0 || ld < d) return comm_fail(SRG_ERR_INVALID, "K=%d d=%d ld=%lld", K, d, (long long)ld);
    const int P = comm->nranks;
    for (int q = 0; q < P; ++q)
        if (row_starts[q + 1] < row_starts[q] || row_starts[0] != 0)
            return comm_fail(SRG_ERR_INVALID, "row_starts must start at 0 and be non-decreasing");
    for (int i = 0; i < n_shards; ++i) {
        const srg_shard_f32& s = shards[i];
        const int r = comm->ranks[i];
        if (s.row0 != row_starts[r] || s.n_rows != row_starts[r + 1] - row_starts[r])
            return comm_fail(SRG_ERR_INVALID, "shard %d (rank %d) rows [%lld, +%lld) != row_starts block",
                             i, r, (long long)s.row0, (long long)s.n_rows);
        if (s.device != comm->devices[i])
            return comm_fail(SRG_ERR_INVALID, "shard %d on device %d, its communicator on %d", i, s.device,
                             comm->devices[i]);
        if (!s.x_full || !s.panels) return comm_fail(SRG_ERR_INVALID, "shard %d: null buffers", i);
        if (s.n_rows > 0 && !s.indptr) return comm_fail(SRG_ERR_INVALID, "shard %d: null indptr", i);
    }
    if (K == 0 || d == 0) return SRG_OK;
    const Rccl* r = nullptr;
    int rc = load_rccl(&r);
    if (rc) return rc;
    DeviceScope scope;
    if ((rc = dist_streams(comm))) return rc;
    auto st = [&](int i) { return static_cast<hipStream_t>(shards[i].stream); };
    // the owner-block split points of every shard's rows (and the check that the rows are sorted:
    // block q must read only rows rank q owns, which have arrived when it runs)
    std::vector<int64_t*> splits(n_shards, nullptr);
    int* bad = nullptr;
    // The split points are read by the span launches on the shard's stream and by their hub rows on
    // the library's side stream.  Every span launch here forks and joins its own hub rows (no
    // HUB_NOJOIN), so the free, enqueued on the shard's stream after the last launch, is already
    // ordered after both; srg_hub_join makes that explicit (a no-op when nothing is pending), so the
    // stream-ordered free never depends on how the launches chained their hub rows.
    auto release = [&]() {
        for (int i = 0; i < n_shards; ++i)
            if (splits[i]) {
                (void)hipSetDevice(shards[i].device);
                (void)srg_hub_join(shards[i].stream);
                (void)hipFreeAsync(splits[i], st(i));
            }
    };
    for (int i = 0; i < n_shards; ++i) {
        const srg_shard_f32& s = shards[i];
        SRG_HIPC(hipSetDevice(s.device));
        // [P + 1] bounds, [P - 1][n_rows] split points, one status word
        const size_t bytes = (size_t)(P + 1) * 8 + (size_t)(P - 1) * (size_t)s.n_rows * 8 + 8;
        if (hipMallocAsync(reinterpret_cast<void**>(&splits[i]), bytes, st(i)) != hipSuccess) {
            release();
            return comm_fail(SRG_ERR_HIP, "shard %d: hipMallocAsync of %zu bytes failed", i, bytes);
        }
        int64_t* bounds = splits[i] + (size_t)(P - 1) * s.n_rows;
        bad = reinterpret_cast<int*>(bounds + P + 1);
        hipError_t e = hipMemcpyAsync(bounds, row_starts, (size_t)(P + 1) * 8, hipMemcpyHostToDevice, st(i));
        if (e == hipSuccess) e = hipMemsetAsync(bad, 0, 4, st(i));
        if (e == hipSuccess && s.n_rows > 0) {
            const unsigned grid = (unsigned)std::min<int64_t>((s.n_rows * 64 + 255) / 256, 1 << 20);
            hipLaunchKernelGGL(k_owner_splits, dim3(grid), dim3(256), 0, st(i), s.indptr, s.indices, s.n_rows, bounds,
                               P, splits[i], bad);
            e = hipGetLastError();
        }
        int flag = 0;
        if (e == hipSuccess) e = hipMemcpyAsync(&flag, bad, 4, hipMemcpyDeviceToHost, st(i));
        if (e == hipSuccess) e = hipStreamSynchronize(st(i));
        if (e != hipSuccess) {
            release();
            return comm_fail(SRG_ERR_HIP, "shard %d: owner splits failed: %s", i, hipGetErrorString(e));
        }
        if (flag) {
            release();
            return comm_fail(SRG_ERR_INVALID, "shard %d: a row's column ids are not sorted (the owner-chunked exchange "
                                              "needs Â's canonical rows, SSRG/operators/utils.py:81-93)", i);
        }
    }
    for (int k = 1; k <= K && !rc; ++k) {
        for (int i = 0; i < n_shards && !rc; ++i) {
            const srg_shard_f32& s = shards[i];
            if (hipSetDevice(s.device) != hipSuccess || hipEventRecord(comm->panel_ready[i], st(i)) != hipSuccess)
                rc = comm_fail(SRG_ERR_HIP, "shard %d: panel event failed", i);
            // the own block is in place at once; the peers' blocks arrive on the pair streams
            else if (s.n_rows && hipMemcpyAsync(s.x_full + (size_t)s.row0 * ld, s.panels[k - 1],
                                                (size_t)s.n_rows * ld * sizeof(float), hipMemcpyDeviceToDevice,
                                                st(i)) != hipSuccess)
                rc = comm_fail(SRG_ERR_HIP, "shard %d: own block copy failed", i);
        }
        if (!rc) rc = dist_exchange(r, comm, shards, n_shards, row_starts, ld, k);
        // block q of every row once rank q's rows are in x_full, ascending q: the chains in CSR order
        for (int i = 0; i < n_shards && !rc; ++i) {
            const srg_shard_f32& s = shards[i];
            const int me = comm->ranks[i];
            if (hipSetDevice(s.device) != hipSuccess) {
                rc = comm_fail(SRG_ERR_HIP, "hipSetDevice(%d) failed", s.device);
                break;
            }
            for (int q = 0; q < P && !rc; ++q) {
                if (q != me && hipStreamWaitEvent(st(i), comm->peer_arrived[i][q], 0) != hipSuccess) {
                    rc = comm_fail(SRG_ERR_HIP, "shard %d: wait for rank %d failed", i, q);
                    break;
                }
                if (s.n_rows == 0) continue;
                const int64_t* beg = q == 0 ? s.indptr : splits[i] + (size_t)(q - 1) * s.n_rows;
                const int64_t* end = q == P - 1 ? s.indptr + 1 : splits[i] + (size_t)q * s.n_rows;
                rc = srg_spmm_span_f32(beg, end, s.indices, s.values, s.n_rows, s.row_order, s.n_hub, s.n_heavy, s.x_full,
                                       ld, s.panels[k], ld, d, q > 0 ? SRG_SPMM_ACCUMULATE : 0u, nullptr, 0, 0.0f, 0,
                                       s.stream);
            }
        }
    }
    // the shards' streams also wait for their last sends (the caller may reuse panel K - 1 after them)
    for (int i = 0; i < n_shards; ++i) {
        (void)hipSetDevice(shards[i].device);
        for (int q = 0; q < P; ++q)
            if (q != comm->ranks[i]) (void)hipStreamWaitEvent(st(i), comm->peer_arrived[i][q], 0);
    }
    release();
    return rc;
}

}  // extern "C"

// ------------------------------------------------------------------------------------------------
// the halo-exchange hop loop (srg_halo.hip builds the plan and the shares)
// ------------------------------------------------------------------------------------------------
namespace {

int64_t view_heavy(const SrgHaloView& V, int d) { return d <= 32 ? V.n_heavy_narrow : V.n_heavy; }

// rows of group g (g == C + 1: the ghost rows of X) that `pl`'s rank sends to / receives from rank q
int64_t send_count(const srg_halo_plan& pl, int g, int q)
{
    return g <= pl.C ? pl.send_counts[g][q] : pl.ghost_send_counts[q];
}
int64_t recv_count(const srg_halo_plan& pl, int g, int q)
{
    return g <= pl.C ? pl.recv_counts[g][q] : pl.ghost_recv_counts[q];
}
int64_t recv_base(const srg_halo_plan& pl, int g)
{
    return pl.rows + (g <= pl.C ? pl.group_offsets[g] : pl.n_recv);
}

// group g's send rows of `panel` (own rows) into the share's send buffer, on `s`; the event marks it
int halo_pack(srg_halo_share* S, int g, const float* panel, int32_t d, hipStream_t s)
{
    const int64_t cnt = S->send_off[g + 1] - S->send_off[g];
    if (cnt > 0) {
        int rc = srg_gather_rows_f32(panel, d, S->plan->rows, S->send_idx[g], cnt, S->sendbuf + S->send_off[g] * d,
                                     d, d, s);
        if (rc) return rc;
    }
    SRG_HIPC(hipEventRecord(S->packed[g], s));
    return SRG_OK;
}

// group g's exchange into the panels `dst` (one per shard): RCCL grouped sends / receives on each
// shard's comm stream, which waits only for that group's pack; or, loopback, device copies
int halo_transport(const Rccl* r, srg_comm* comm, srg_halo_share* const* shares, int n, int g,
                   float* const* dst, int32_t d)
{
    const int P = comm->nranks;
    if (comm->loopback) {
        hipStream_t L = comm->lb_stream;
        for (int i = 0; i < n; ++i) SRG_HIPC(hipStreamWaitEvent(L, shares[i]->packed[g], 0));
        for (int q = 0; q < n; ++q) {
            const srg_halo_plan& pq = *shares[q]->plan;
            int64_t roff = recv_base(pq, g);
            for (int s = 0; s < P; ++s) {
                if (s == q) continue;
                const int64_t cnt = recv_count(pq, g, s);
                if (cnt > 0) {
                    const srg_halo_plan& ps = *shares[s]->plan;
                    int64_t soff = shares[s]->send_off[g];
                    for (int t = 0; t < q; ++t)
                        if (t != s) soff += send_count(ps, g, t);
                    SRG_HIPC(hipMemcpyAsync(dst[q] + roff * d, shares[s]->sendbuf + soff * d,
                                            (size_t)cnt * d * sizeof(float), hipMemcpyDeviceToDevice, L));
                }
                roff += cnt;
            }
        }
        return SRG_OK;
    }
    for (int i = 0; i < n; ++i) {
        SRG_HIPC(hipSetDevice(shares[i]->device));
        SRG_HIPC(hipStreamWaitEvent(shares[i]->comm_stream, shares[i]->packed[g], 0));
    }
    SRG_NCCL(r, r->GroupStart());
    int rc = SRG_OK;
    for (int i = 0; i < n && !rc; ++i) {
        srg_halo_share* S = shares[i];
        const srg_halo_plan& pl = *S->plan;
        const int me = comm->ranks[i];
        int64_t soff = S->send_off[g], roff = recv_base(pl, g);
        for (int q = 0; q < P && !rc; ++q) {
            if (q == me) continue;
            const int64_t sc = send_count(pl, g, q), rcn = recv_count(pl, g, q);
            ncclResult_t e = ncclSuccess;
            if (sc > 0) e = r->Send(S->sendbuf + soff * d, (size_t)sc * d, ncclFloat32, q, comm->comms[i], S->comm_stream);
            if (e == ncclSuccess && rcn > 0)
                e = r->Recv(dst[i] + roff * d, (size_t)rcn * d, ncclFloat32, q, comm->comms[i], S->comm_stream);
            if (e != ncclSuccess) rc = comm_fail(SRG_ERR_HIP, "ncclSend / ncclRecv failed: %s", r->GetErrorString(e));
            soff += sc;
            roff += rcn;
        }
    }
    // every exit closes the group (RCCL's group state is thread-local and shared with torch)
    const ncclResult_t ge = r->GroupEnd();
    if (rc) return rc;
    if (ge != ncclSuccess) return comm_fail(SRG_ERR_HIP, "ncclGroupEnd failed: %s", r->GetErrorString(ge));
    return SRG_OK;
}

// Before a share's first exchange over RCCL: every rank sends each peer what it will send it -- the
// rows of every group and of X's ghost rows, plus (n, nnz) of the plan's graph -- and checks that
// against what it expects to receive.  Plans built with different arguments (chunks, thresholds, ghost
// caps, graphs) then fail with SRG_ERR_INVALID instead of hanging in ncclGroupEnd or filling the halo
// with the wrong rows.  Two small grouped exchanges and two host syncs per share, once: first a
// fixed-size header (groups C, n, nnz, ranks P) -- its length never depends on the plan, so ranks whose
// plans have different chunk counts still exchange matching messages and all fail on the mismatch
// (every rank that differs from any rank sees a difference: a != b means no rank equals both) -- then,
// only when every header agrees, the C + 2 per-group counts.
constexpr int kCountHeader = 4;

// one grouped exchange of `len` int64 per peer: buf[i] holds [P][len] to send, then [P][len] received
int exchange_words(const Rccl* r, srg_comm* comm, srg_halo_share* const* shares, int n, const std::vector<int64_t*>& buf,
                   const std::vector<std::vector<int64_t>>& mine, int len, std::vector<std::vector<int64_t>>& theirs)
{
    const int P = comm->nranks;
    for (int i = 0; i < n; ++i)
        if (hipSetDevice(shares[i]->device) != hipSuccess ||
            hipMemcpy(buf[i], mine[i].data(), (size_t)P * len * sizeof(int64_t), hipMemcpyHostToDevice) != hipSuccess)
            return comm_fail(SRG_ERR_HIP, "share %d: count upload failed", i);
    if (r->GroupStart() != ncclSuccess) return comm_fail(SRG_ERR_HIP, "ncclGroupStart failed");
    int rc = SRG_OK;
    for (int i = 0; i < n && !rc; ++i) {
        const int me = comm->ranks[i];
        for (int q = 0; q < P && !rc; ++q) {
            if (q == me) continue;
            ncclResult_t e = r->Send(buf[i] + (size_t)q * len, len, ncclInt64, q, comm->comms[i], shares[i]->comm_stream);
            if (e == ncclSuccess)
                e = r->Recv(buf[i] + (size_t)(P + q) * len, len, ncclInt64, q, comm->comms[i], shares[i]->comm_stream);
            if (e != ncclSuccess) rc = comm_fail(SRG_ERR_HIP, "count exchange failed: %s", r->GetErrorString(e));
        }
    }
    const ncclResult_t ge = r->GroupEnd();
    if (!rc && ge != ncclSuccess) rc = comm_fail(SRG_ERR_HIP, "count exchange: ncclGroupEnd failed: %s", r->GetErrorString(ge));
    theirs.assign(n, std::vector<int64_t>((size_t)P * len, 0));
    for (int i = 0; i < n && !rc; ++i)
        if (hipSetDevice(shares[i]->device) != hipSuccess || hipStreamSynchronize(shares[i]->comm_stream) != hipSuccess ||
            hipMemcpy(theirs[i].data(), buf[i] + (size_t)P * len, (size_t)P * len * sizeof(int64_t), hipMemcpyDeviceToHost) !=
                hipSuccess)
            rc = comm_fail(SRG_ERR_HIP, "share %d: count exchange readback failed", i);
    return rc;
}

int verify_counts(const Rccl* r, srg_comm* comm, srg_halo_share* const* shares, int n)
{
    bool all = true;
    for (int i = 0; i < n; ++i) all &= shares[i]->counts_verified;
    if (all) return SRG_OK;
    const int P = comm->nranks;
    int cmax = 0;
    for (int i = 0; i < n; ++i) cmax = std::max(cmax, shares[i]->plan->C);
    const int NG = std::max(cmax + 2, kCountHeader);   // words per peer: the buffers fit either exchange
    std::vector<int64_t*> buf(n, nullptr);
    auto release = [&]() {
        for (int i = 0; i < n; ++i)
            if (buf[i]) {
                (void)hipSetDevice(shares[i]->device);
                (void)hipFree(buf[i]);
            }
    };
    for (int i = 0; i < n; ++i)
        if (hipSetDevice(shares[i]->device) != hipSuccess ||
            hipMalloc(reinterpret_cast<void**>(&buf[i]), (size_t)2 * P * NG * sizeof(int64_t)) != hipSuccess) {
            release();
            return comm_fail(SRG_ERR_HIP, "share %d: count buffers failed", i);
        }
    // 1: the header, kCountHeader words per peer whatever the plan
    std::vector<std::vector<int64_t>> mine(n), theirs;
    for (int i = 0; i < n; ++i) {
        const srg_halo_plan& pl = *shares[i]->plan;
        mine[i].assign((size_t)P * kCountHeader, 0);
        for (int q = 0; q < P; ++q) {
            int64_t* h = mine[i].data() + (size_t)q * kCountHeader;
            h[0] = pl.C;
            h[1] = pl.n;
            h[2] = pl.nnz_total;
            h[3] = P;
        }
    }
    int rc = exchange_words(r, comm, shares, n, buf, mine, kCountHeader, theirs);
    for (int i = 0; i < n && !rc; ++i) {
        const srg_halo_plan& pl = *shares[i]->plan;
        for (int q = 0; q < P && !rc; ++q) {
            if (q == comm->ranks[i]) continue;
            const int64_t* t = theirs[i].data() + (size_t)q * kCountHeader;
            if (t[1] != pl.n || t[2] != pl.nnz_total)
                rc = comm_fail(SRG_ERR_INVALID, "rank %d's plan is of a graph with n=%lld nnz=%lld, rank %d's of n=%lld "
                               "nnz=%lld", q, (long long)t[1], (long long)t[2], comm->ranks[i], (long long)pl.n,
                               (long long)pl.nnz_total);
            else if (t[0] != pl.C || t[3] != P)
                rc = comm_fail(SRG_ERR_INVALID, "plans disagree: rank %d's plan has %lld row chunks over %lld ranks, rank "
                               "%d's %d over %d (build every rank's plan with the same arguments)", q, (long long)t[0],
                               (long long)t[3], comm->ranks[i], pl.C, P);
        }
    }
    // 2: the per-group counts (every plan has the same C now)
    if (!rc) {
        const int C = shares[0]->plan->C, len = C + 2;
        for (int i = 0; i < n; ++i) {
            const srg_halo_plan& pl = *shares[i]->plan;
            mine[i].assign((size_t)P * len, 0);
            for (int q = 0; q < P; ++q)
                for (int g = 0; g <= C + 1; ++g) mine[i][(size_t)q * len + g] = send_count(pl, g, q);
        }
        rc = exchange_words(r, comm, shares, n, buf, mine, len, theirs);
        for (int i = 0; i < n && !rc; ++i) {
            const srg_halo_plan& pl = *shares[i]->plan;
            for (int q = 0; q < P && !rc; ++q) {
                if (q == comm->ranks[i]) continue;
                const int64_t* t = theirs[i].data() + (size_t)q * len;
                for (int g = 0; g <= C + 1 && !rc; ++g)
                    if (t[g] != recv_count(pl, g, q))
                        rc = comm_fail(SRG_ERR_INVALID, "plans disagree: rank %d sends %lld rows of group %d to rank %d, "
                                       "which expects %lld (build every rank's plan with the same arguments)", q,
                                       (long long)t[g], g, comm->ranks[i], (long long)recv_count(pl, g, q));
            }
        }
    }
    release();
    if (!rc)
        for (int i = 0; i < n; ++i) shares[i]->counts_verified = true;
    return rc;
}

// every shard's stream waits for the exchanges issued so far (on the device, not the host)
int halo_finish(srg_comm* comm, srg_halo_share* const* shares, int n, void* const* streams)
{
    if (comm->loopback) {
        SRG_HIPC(hipEventRecord(comm->lb_done, comm->lb_stream));
        for (int i = 0; i < n; ++i)
            SRG_HIPC(hipStreamWaitEvent(streams ? static_cast<hipStream_t>(streams[i]) : nullptr, comm->lb_done, 0));
        return SRG_OK;
    }
    for (int i = 0; i < n; ++i) {
        SRG_HIPC(hipSetDevice(shares[i]->device));
        SRG_HIPC(hipEventRecord(shares[i]->comm_done, shares[i]->comm_stream));
        SRG_HIPC(hipStreamWaitEvent(streams ? static_cast<hipStream_t>(streams[i]) : nullptr, shares[i]->comm_done, 0));
    }
    return SRG_OK;
}

}  // namespace

extern "C" {

int srg_halo_propagate_f32(srg_comm* comm, srg_halo_share* const* shares, int n_shards, float* const* const* panels,
                           int64_t ld, int32_t d, int32_t K, uint32_t flags, void* const* streams)
{
    if (!comm || !shares || !panels) return comm_fail(SRG_ERR_INVALID, "null argument");
    const int P = comm->nranks;
    const int local = comm->loopback ? P : (int)comm->comms.size();
    if (n_shards != local) return comm_fail(SRG_ERR_INVALID, "%d shares for %d local ranks", n_shards, local);
    if (K < 0 || d < 0) return comm_fail(SRG_ERR_INVALID, "K=%d d=%d", K, d);
    if (ld != d) return comm_fail(SRG_ERR_INVALID, "ld=%lld != d=%d: the halo rows are contiguous exchange buffers",
                                  (long long)ld, d);
    int C = -1;
    for (int i = 0; i < n_shards; ++i) {
        const srg_halo_share* S = shares[i];
        if (!S || !S->plan || !panels[i]) return comm_fail(SRG_ERR_INVALID, "share %d: null share or panels", i);
        const srg_halo_plan& pl = *S->plan;
        if (pl.P != P || pl.p != comm->ranks[i])
            return comm_fail(SRG_ERR_INVALID, "share %d is rank %d of %d, its communicator rank %d of %d", i, pl.p, pl.P,
                             comm->ranks[i], P);
        if (S->device != comm->devices[i])
            return comm_fail(SRG_ERR_INVALID, "share %d on device %d, its communicator on %d", i, S->device, comm->devices[i]);
        if (d > S->d_cap) return comm_fail(SRG_ERR_INVALID, "d=%d > the share's d_max=%lld", d, (long long)S->d_cap);
        if (C >= 0 && pl.C != C) return comm_fail(SRG_ERR_INVALID, "shares with different chunk counts");
        C = pl.C;
        for (int k = 0; k <= K; ++k)
            if (!panels[i][k] && d > 0) return comm_fail(SRG_ERR_INVALID, "share %d: panels[%d] is null", i, k);
    }
    if (comm->loopback)    // the plans of the in-process ranks must agree on every count
        for (int g = 0; g <= C + 1; ++g)
            for (int q = 0; q < P; ++q)
                for (int s = 0; s < P; ++s)
                    if (s != q && recv_count(*shares[q]->plan, g, s) != send_count(*shares[s]->plan, g, q))
                        return comm_fail(SRG_ERR_INVALID, "group %d: rank %d receives %lld rows from %d, which sends %lld",
                                         g, q, (long long)recv_count(*shares[q]->plan, g, s), s,
                                         (long long)send_count(*shares[s]->plan, g, q));
    if (K == 0 || d == 0) return SRG_OK;
    const Rccl* r = nullptr;
    DeviceScope scope;
    if (!comm->loopback) {
        int rc = load_rccl(&r);
        if (!rc) rc = verify_counts(r, comm, shares, n_shards);
        if (rc) return rc;
    }
    const int G = C + 1;
    auto st = [&](int i) { return streams ? static_cast<hipStream_t>(streams[i]) : nullptr; };
    std::vector<float*> dst(n_shards);
    auto panel_k = [&](int k) {
        for (int i = 0; i < n_shards; ++i) dst[i] = panels[i][k];
        return dst.data();
    };
    int rc = SRG_OK;
    // hop 0's halo (received rows by group, then the ghost rows), unless the caller filled it
    if (!(flags & SRG_HALO_X_HALO_FILLED)) {
        for (int g = 0; g <= G; ++g) {
            for (int i = 0; i < n_shards; ++i) {
                SRG_HIPC(hipSetDevice(shares[i]->device));
                if ((rc = halo_pack(shares[i], g, panels[i][0], d, st(i)))) return rc;
            }
            if ((rc = halo_transport(r, comm, shares, n_shards, g, panel_k(0), d))) return rc;
        }
        if ((rc = halo_finish(comm, shares, n_shards, streams))) return rc;
    }
    for (int k = 1; k <= K; ++k) {
        const bool ex = k < K;       // the last hop's halo is never read
        auto launch = [&](int i, int v, uint32_t f) -> int {
            const srg_halo_share* S = shares[i];
            const SrgHaloView& V = S->plan->views[v];
            if (V.n == 0) return SRG_OK;
            return srg_spmm_csr_f32(S->lip, S->lix, S->lvv, V.n, S->orders[v], V.n_hub, view_heavy(V, d),
                                    panels[i][k - 1], ld, panels[i][k], ld, d, f, st(i));
        };
        // the hub group forked onto the library's side stream, beside the chunks
        for (int i = 0; i < n_shards; ++i) {
            SRG_HIPC(hipSetDevice(shares[i]->device));
            if ((rc = launch(i, C, SRG_SPMM_HUB_NOJOIN))) return rc;
        }
        // a row chunk: one launch, or its column blocks in order (the share's, when d asks for as many)
        auto chunk = [&](int i, int c) -> int {
            const srg_halo_share* S = shares[i];
            const SrgHaloBlocks& Kb = S->blocks;
            if (Kb.B < 2 || (!Kb.forced && srg_halo_col_blocks(S->plan->rows + S->plan->halo, d) != Kb.B))
                return launch(i, c, 0);
            const uint32_t u2 = d >= 128 ? SRG_SPMM_PACKED_U2 : 0u;
            for (int b = 0; b < Kb.B; ++b) {
                const SrgHaloView& V = Kb.views[c][b];
                if (V.n == 0) continue;
                const int e = srg_spmm_span_f32(Kb.bounds[b], Kb.bounds[b + 1], S->lix, S->lvv, V.n, Kb.orders[c][b], 0,
                                                view_heavy(V, d), panels[i][k - 1], ld, panels[i][k], ld, d,
                                                (b > 0 ? SRG_SPMM_ACCUMULATE : 0u) | u2, nullptr, 0, 0.0f, 0, st(i));
                if (e) return e;
            }
            return SRG_OK;
        };
        for (int c = 0; c < C; ++c) {
            for (int i = 0; i < n_shards; ++i) {
                SRG_HIPC(hipSetDevice(shares[i]->device));
                if ((rc = chunk(i, c))) return rc;
                if (ex && (rc = halo_pack(shares[i], c, panels[i][k], d, st(i)))) return rc;
            }
            if (ex && (rc = halo_transport(r, comm, shares, n_shards, c, panel_k(k), d))) return rc;
        }
        for (int i = 0; i < n_shards; ++i) {
            SRG_HIPC(hipSetDevice(shares[i]->device));
            if (ex && (rc = launch(i, G, 0))) return rc;            // the ghost rows into their halo slots
            if (shares[i]->plan->views[C].n && (rc = srg_hub_join(st(i)))) return rc;
            if (ex && (rc = halo_pack(shares[i], C, panels[i][k], d, st(i)))) return rc;
        }
        if (ex) {
            if ((rc = halo_transport(r, comm, shares, n_shards, C, panel_k(k), d))) return rc;
            if ((rc = halo_finish(comm, shares, n_shards, streams))) return rc;
        }
    }
    return SRG_OK;
}

}  // extern "C"
