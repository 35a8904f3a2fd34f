// srg_comm.hip -- communicator lifecycle and the row-partitioned K-hop propagation over RCCL, for C / C++
// hosts (the Python package drives the same kernels through torch.distributed,
// srgnn/dist.py).
//
// Partition: rank r owns rows [row_starts[r], row_starts[r+1]) of Â (a 1-D, contiguous row block with
// global column ids) and the same rows of every hop panel.  Per hop, every rank's block of the previous
// panel is exchanged with grouped ncclSend / ncclRecv (variable block sizes, every peer at once: a
// direct all-gather over xGMI's point-to-point links), the own block is copied device-to-device, and the
// rank's rows are multiplied by srg_spmm_csr_f32 on the gathered panel.  Each row's fma chain is the
// one-GPU chain, so every hop is bitwise the one-GPU hop.
//
// RCCL is loaded at run time (dlopen, RTLD_LOCAL): a process that already holds an RCCL (PyTorch's) keeps
// using that one, and the library itself has no link-time dependency on it.  SRGNN_RCCL_LIB names a
// specific librccl.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <dlfcn.h>

#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <vector>

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
};

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

int srg_comm_destroy(srg_comm* comm)
{
    if (!comm) return SRG_OK;
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

// The sends and receives of hop k's exchange (inside the caller's GroupStart / GroupEnd bracket).
static int group_sends(const Rccl* r, srg_comm* comm, const srg_shard_f32* shards, int n_shards,
                       const int64_t* row_starts, int64_t ld, int k, int P)
{
    for (int i = 0; i < n_shards; ++i) {
        const srg_shard_f32& s = shards[i];
        const int me = comm->ranks[i];
        SRG_HIPC(hipSetDevice(s.device));
        hipStream_t st = static_cast<hipStream_t>(s.stream);
        for (int q = 0; q < P; ++q) {
            if (q == me) continue;
            const size_t nq = (size_t)(row_starts[q + 1] - row_starts[q]) * (size_t)ld;
            const size_t nme = (size_t)s.n_rows * (size_t)ld;
            if (nme) SRG_NCCL(r, r->Send(s.panels[k - 1], nme, ncclFloat32, q, comm->comms[i], st));
            if (nq) SRG_NCCL(r, r->Recv(s.x_full + (size_t)row_starts[q] * ld, nq, ncclFloat32, q, comm->comms[i], st));
        }
    }
    return SRG_OK;
}

int srg_dist_propagate_khop_f32(srg_comm* comm, const srg_shard_f32* shards, int n_shards,
                                const int64_t* row_starts, int64_t ld, int32_t d, int32_t K)
{
    if (!comm || !shards || !row_starts) return comm_fail(SRG_ERR_INVALID, "null argument");
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
    }
    if (K == 0 || d == 0) return SRG_OK;
    const Rccl* r = nullptr;
    int rc = load_rccl(&r);
    if (rc) return rc;
    DeviceScope scope;
    const size_t esz = sizeof(float);
    for (int k = 1; k <= K; ++k) {
        // exchange: every rank's block of panel k-1 into every other rank's gathered panel
        SRG_NCCL(r, r->GroupStart());
        // every exit from the bracket closes the group: an error inside it must not leave RCCL's
        // thread-local group open (later RCCL calls of the process, torch's included, would be
        // folded into it); the first error is the one returned
        rc = group_sends(r, comm, shards, n_shards, row_starts, ld, k, P);
        const ncclResult_t ge = r->GroupEnd();
        if (rc) return rc;
        if (ge != ncclSuccess) return comm_fail(SRG_ERR_HIP, "ncclGroupEnd failed: %s", r->GetErrorString(ge));
        for (int i = 0; i < n_shards; ++i) {
            const srg_shard_f32& s = shards[i];
            SRG_HIPC(hipSetDevice(s.device));
            hipStream_t st = static_cast<hipStream_t>(s.stream);
            if (s.n_rows)
                SRG_HIPC(hipMemcpyAsync(s.x_full + (size_t)s.row0 * ld, s.panels[k - 1], (size_t)s.n_rows * ld * esz,
                                        hipMemcpyDeviceToDevice, st));
            int e = srg_spmm_csr_f32(s.indptr, s.indices, s.values, s.n_rows, s.row_order, s.n_hub, s.n_heavy,
                                     s.x_full, ld, s.panels[k], ld, d, 0, s.stream);
            if (e) return e;
        }
    }
    return SRG_OK;
}

}  // extern "C"
