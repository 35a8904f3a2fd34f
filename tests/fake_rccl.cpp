// fake_rccl.cpp -- TEST-ONLY stand-in for librccl's point-to-point API, loaded by libsrgnn_hip through
// SRGNN_RCCL_LIB.  It lets one process on ONE GPU run the library's RCCL code paths (srg_comm.hip:
// srg_dist_propagate_khop_f32, halo_transport's RCCL branch) with P > 1 ranks, which real RCCL refuses
// on a single device ("Duplicate GPU detected").  Never part of the product library.
//
// Semantics (a subset of NCCL 2.x / RCCL p2p):
//   * ncclCommInitAll(comms, n, devs) makes n communicators of one world (ranks 0..n-1, devices as
//     given; repeated devices allowed); ncclCommInitRank only for nranks == 1;
//   * ncclSend / ncclRecv are queued; at the end of the outermost group (or at once, outside one)
//     every queued receive is matched with the oldest pending send of (src -> dst) and vice versa;
//     a matched pair becomes a device copy on the RECEIVER's stream after the sender's stream point
//     (an event), and the sender's stream then waits for the copy -- as if each stream's p2p kernel
//     completed with the transfer;
//   * counts or types that disagree, or operations left unmatched at the end of a group, return
//     ncclInvalidUsage (real RCCL would hang): the tests see a plan mismatch as an error.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdio>
#include <cstring>
#include <deque>
#include <map>
#include <mutex>
#include <utility>
#include <vector>

namespace {

struct World;
struct Comm {
    int rank = 0, dev = 0;
    World* world = nullptr;
};
struct World {
    int n = 0;
    int alive = 0;
};

struct Op {
    bool send = false;
    void* buf = nullptr;
    size_t count = 0;
    ncclDataType_t type = ncclFloat32;
    int me = 0, peer = 0;
    World* world = nullptr;
    int dev = 0;
    hipStream_t stream = nullptr;
};

std::mutex g_mu;
thread_local int g_depth = 0;
thread_local std::vector<Op> g_queued;
// unmatched operations of earlier groups, per (world, src, dst)
std::map<std::pair<World*, std::pair<int, int>>, std::deque<Op>> g_sends, g_recvs;
std::vector<std::pair<int, hipEvent_t>> g_events;   // (device, event): destroyed with the last communicator
int g_worlds = 0;

size_t type_size(ncclDataType_t t)
{
    switch (t) {
        case ncclInt8: case ncclUint8: return 1;
        case ncclFloat16: case ncclBfloat16: return 2;
        case ncclInt32: case ncclUint32: case ncclFloat32: return 4;
        case ncclInt64: case ncclUint64: case ncclFloat64: return 8;
        default: return 0;
    }
}

ncclResult_t transfer(const Op& s, const Op& r)
{
    if (s.count != r.count || s.type != r.type) {
        fprintf(stderr, "fake_rccl: rank %d sends %zu x type %d to %d, which receives %zu x type %d\n", s.me, s.count,
                (int)s.type, r.me, r.count, (int)r.type);
        return ncclInvalidUsage;
    }
    const size_t bytes = s.count * type_size(s.type);
    if (!bytes) return ncclSuccess;
    hipEvent_t sent = nullptr, done = nullptr;
    if (hipSetDevice(s.dev) != hipSuccess || hipEventCreateWithFlags(&sent, hipEventDisableTiming) != hipSuccess ||
        hipEventRecord(sent, s.stream) != hipSuccess)
        return ncclUnhandledCudaError;
    if (hipSetDevice(r.dev) != hipSuccess || hipStreamWaitEvent(r.stream, sent, 0) != hipSuccess ||
        hipMemcpyAsync(r.buf, s.buf, bytes, hipMemcpyDeviceToDevice, r.stream) != hipSuccess ||
        hipEventCreateWithFlags(&done, hipEventDisableTiming) != hipSuccess || hipEventRecord(done, r.stream) != hipSuccess)
        return ncclUnhandledCudaError;
    if (hipSetDevice(s.dev) != hipSuccess || hipStreamWaitEvent(s.stream, done, 0) != hipSuccess)
        return ncclUnhandledCudaError;
    g_events.push_back({s.dev, sent});
    g_events.push_back({r.dev, done});
    return ncclSuccess;
}

ncclResult_t flush()
{
    std::lock_guard<std::mutex> lock(g_mu);
    int prev = 0;
    (void)hipGetDevice(&prev);
    ncclResult_t rc = ncclSuccess;
    for (const Op& op : g_queued) {
        const auto key = op.send ? std::make_pair(op.world, std::make_pair(op.me, op.peer))
                                 : std::make_pair(op.world, std::make_pair(op.peer, op.me));
        auto& other = op.send ? g_recvs[key] : g_sends[key];
        if (!other.empty()) {
            const Op o = other.front();
            other.pop_front();
            const ncclResult_t e = op.send ? transfer(op, o) : transfer(o, op);
            if (e != ncclSuccess && rc == ncclSuccess) rc = e;
        } else {
            (op.send ? g_sends[key] : g_recvs[key]).push_back(op);
        }
    }
    g_queued.clear();
    // a group must be self-contained in this single-process world: nothing may stay pending
    for (auto* m : {&g_sends, &g_recvs})
        for (auto& kv : *m)
            if (!kv.second.empty()) {
                fprintf(stderr, "fake_rccl: %zu unmatched %s from rank %d to rank %d at the end of a group\n",
                        kv.second.size(), m == &g_sends ? "sends" : "receives", kv.first.second.first,
                        kv.first.second.second);
                kv.second.clear();
                if (rc == ncclSuccess) rc = ncclInvalidUsage;
            }
    (void)hipSetDevice(prev);
    return rc;
}

ncclResult_t enqueue(bool send, const void* buf, size_t count, ncclDataType_t type, int peer, ncclComm_t comm,
                     hipStream_t stream)
{
    Comm* c = reinterpret_cast<Comm*>(comm);
    if (!c || peer < 0 || peer >= c->world->n || peer == c->rank || !type_size(type)) return ncclInvalidArgument;
    Op op;
    op.send = send;
    op.buf = const_cast<void*>(buf);
    op.count = count;
    op.type = type;
    op.me = c->rank;
    op.peer = peer;
    op.world = c->world;
    op.dev = c->dev;
    op.stream = stream;
    g_queued.push_back(op);
    return g_depth > 0 ? ncclSuccess : flush();
}

}  // namespace

extern "C" {

ncclResult_t ncclGetUniqueId(ncclUniqueId* id)
{
    if (!id) return ncclInvalidArgument;
    memset(id, 0, sizeof(*id));
    return ncclSuccess;
}

ncclResult_t ncclCommInitAll(ncclComm_t* comms, int ndev, const int* devlist)
{
    if (!comms || ndev < 1) return ncclInvalidArgument;
    World* w = new World();
    {
        std::lock_guard<std::mutex> lock(g_mu);
        ++g_worlds;
    }
    w->n = ndev;
    w->alive = ndev;
    for (int i = 0; i < ndev; ++i) {
        Comm* c = new Comm();
        c->rank = i;
        c->dev = devlist ? devlist[i] : i;
        c->world = w;
        comms[i] = reinterpret_cast<ncclComm_t>(c);
    }
    return ncclSuccess;
}

ncclResult_t ncclCommInitRank(ncclComm_t* comm, int nranks, ncclUniqueId, int rank)
{
    if (!comm || nranks != 1 || rank != 0) return ncclInvalidUsage;   // one process hosts the whole world
    int dev = 0;
    (void)hipGetDevice(&dev);
    return ncclCommInitAll(comm, 1, &dev);
}

ncclResult_t ncclCommDestroy(ncclComm_t comm)
{
    Comm* c = reinterpret_cast<Comm*>(comm);
    if (!c) return ncclInvalidArgument;
    World* w = c->world;
    delete c;
    if (--w->alive == 0) {
        delete w;
        std::lock_guard<std::mutex> lock(g_mu);
        if (--g_worlds == 0) {
            for (auto& e : g_events) {
                (void)hipSetDevice(e.first);
                (void)hipEventSynchronize(e.second);
                (void)hipEventDestroy(e.second);
            }
            g_events.clear();
        }
    }
    return ncclSuccess;
}

ncclResult_t ncclGroupStart()
{
    ++g_depth;
    return ncclSuccess;
}

ncclResult_t ncclGroupEnd()
{
    if (g_depth <= 0) return ncclInvalidUsage;
    return --g_depth == 0 ? flush() : ncclSuccess;
}

ncclResult_t ncclSend(const void* buf, size_t count, ncclDataType_t type, int peer, ncclComm_t comm, hipStream_t stream)
{
    return enqueue(true, buf, count, type, peer, comm, stream);
}

ncclResult_t ncclRecv(void* buf, size_t count, ncclDataType_t type, int peer, ncclComm_t comm, hipStream_t stream)
{
    return enqueue(false, buf, count, type, peer, comm, stream);
}

const char* ncclGetErrorString(ncclResult_t r)
{
    switch (r) {
        case ncclSuccess: return "no error (fake_rccl)";
        case ncclInvalidArgument: return "invalid argument (fake_rccl)";
        case ncclInvalidUsage: return "invalid usage: unmatched or mismatched send / receive (fake_rccl)";
        case ncclUnhandledCudaError: return "HIP call failed (fake_rccl)";
        default: return "error (fake_rccl)";
    }
}

}  // extern "C"
