// srg_halo.hip -- the halo-exchange partition for C / C++ hosts: the host planner that derives rank p's
// share from the GLOBAL CSR (the same plan srgnn/dist.py HaloPartitionedOperator builds with torch,
// restated in C++), and the device share (local CSR, schedules, send lists, send buffer) the executor
// srg_halo_propagate_f32 (srg_comm.hip) runs the hops on.  SURVEY.md §8(b) item 5 / §8(e).
//
// The plan, deterministic from the global operator and identical on every rank (no messages):
//   * rows: rank p owns the nnz-balanced row block [starts[p], starts[p+1]);
//   * groups: each owner's rows are cut into C nnz-balanced contiguous chunks, except its hub rows
//     (longer than its hub threshold), which form group C; the exchange runs group by group in
//     that order, each group's rows sent as soon as its launch is done;
//   * halos: rank q needs the distinct remote columns of its rows, ordered by (group on the owner,
//     owner, id), so every sender knows what to send and in which order;
//   * ghost rows: a halo row of at most ghost_max_degree entries whose columns all lie in q's own
//     rows or halo is computed on q every hop (the same CSR row in the same order: the same bits)
//     instead of received; exchanged once, with X;
//   * local panel: [own rows | received halo rows by (group, source, id) | ghosts by (source, id)],
//     and the local CSR (own rows, then empty rows for the received halo, then the ghost rows) with
//     its column ids remapped into it -- every row keeps its entries in CSR order, so every output
//     element is the one-GPU fma chain: the N-rank hops are bitwise the one-GPU hops.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <thread>
#include <vector>

#include "srg_halo_internal.h"
#include "srgnn_hip.h"

extern "C" void srg_set_error(int code, const char* msg);   // srg_spmm.hip: thread-local srg_last_error
extern "C" void srg_clear_error(void);

namespace {

int hfail(int code, const char* fmt, ...)
{
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    srg_set_error(code, buf);
    return code;
}

#define SRG_HALO_HIP(expr)                                                                       \
    do {                                                                                         \
        hipError_t e_ = (expr);                                                                  \
        if (e_ != hipSuccess)                                                                    \
            return hfail(SRG_ERR_HIP, "%s failed: %s", #expr, hipGetErrorString(e_));            \
    } while (0)

// srgnn.dist.balanced_row_starts: row bounds s_0 = 0 <= ... <= s_parts = n with about equal nonzeros;
// ip holds n + 1 row pointers, `base` is ip's value at the first row (a block of a larger CSR)
std::vector<int64_t> balanced(const int64_t* ip, int64_t n, int parts, int64_t base)
{
    std::vector<int64_t> s(parts + 1);
    const int64_t nnz = ip[n] - base;
    for (int q = 0; q <= parts; ++q) {
        const int64_t target = nnz * q / parts + base;
        int64_t i = std::lower_bound(ip, ip + n + 1, target) - ip;   // first pointer >= target
        s[q] = std::min<int64_t>(std::max<int64_t>(i, 0), n);
    }
    s[0] = 0;
    s[parts] = n;
    for (int q = 1; q <= parts; ++q) s[q] = std::max(s[q], s[q - 1]);
    return s;
}

// csr.auto_hub_threshold / auto_heavy_threshold
int64_t auto_hub(int64_t nnz, int launches) { return std::max<int64_t>(2048, nnz / (1024 * std::max(1, launches))); }
int64_t auto_heavy(int64_t nnz, int launches) { return std::max<int64_t>(96, nnz / (100000 * std::max(1, launches))); }
constexpr int64_t kNarrowHeavy = 32;   // csr.NARROW_HEAVY_THRESHOLD
constexpr int64_t kHaloHeavyMin = 192; // dist.HALO_HEAVY_MIN: the chunks' slice-wave threshold floor

// rows sorted by decreasing degree, ties in the given order (torch.sort(..., descending, stable))
void sort_by_degree(std::vector<int32_t>& rows, const std::vector<int64_t>& deg_of)
{
    std::stable_sort(rows.begin(), rows.end(), [&](int32_t a, int32_t b) { return deg_of[a] > deg_of[b]; });
}

// rows of at most this many entries run whole in block 0 (= srgnn.csr.BLOCK_WHOLE_MAX)
constexpr int64_t kBlockWholeMax = 48;

// the automatic ghost cap (ghost_max_degree = SRG_HALO_AUTO): candidates, the scan limit and the
// modelled gather rate (products at P = 2: 63.1 M nonzeros x 512 B in 3.85 ms); DESIGN.md §7
constexpr int kGhostScanMax = 64;
constexpr int kGhostCaps[] = {0, 1, 2, 3, 4, 6, 8, 12, 16, 24, 32, 48, 64};
constexpr int kNumGhostCaps = (int)(sizeof(kGhostCaps) / sizeof(kGhostCaps[0]));
constexpr double kGhostGatherBps = 8.4e12;
constexpr double kGhostLinkBps = 64e9;

// host threads for the planner's loops (the GPU boxes grant a job 16 CPUs)
int plan_threads()
{
    return (int)std::max(1u, std::min<unsigned>(std::thread::hardware_concurrency(), 16u));
}

// f(lo, hi) over [0, count) in contiguous pieces, one per thread
template <typename F>
void parallel_ranges(int64_t count, F f)
{
    const int nt = count < (1 << 16) ? 1 : plan_threads();
    if (nt == 1) { f((int64_t)0, count); return; }
    std::vector<std::thread> th;
    for (int t = 0; t < nt; ++t) {
        const int64_t lo = count * t / nt, hi = count * (t + 1) / nt;
        th.emplace_back([=, &f]() { f(lo, hi); });
    }
    for (auto& x : th) x.join();
}

void free_blocks(SrgHaloBlocks& K)
{
    for (auto* sp : K.splits) (void)hipFree(sp);
    for (auto& oc : K.orders)
        for (auto* o : oc) (void)hipFree(o);
    K = SrgHaloBlocks();
}

// The chunks' column blocks of share S (SrgHaloBlocks): split points on the host from the entries'
// global column ids (the binary search of srg_csr_col_splits), per (chunk, block) schedules sorted by
// span length (stable, from the chunk's degree order), uploaded.
int build_blocks(srg_halo_share* S, int B)
{
    const srg_halo_plan& pl = *S->plan;
    SrgHaloBlocks& K = S->blocks;
    const int64_t rows = pl.rows;
    const int C = pl.C;
    const int64_t whole_max = kBlockWholeMax;
    std::vector<std::vector<int64_t>> sp((size_t)B - 1, std::vector<int64_t>((size_t)rows));
    auto glob = [&](int32_t l) -> int64_t { return l < rows ? pl.r0 + l : pl.halo_ids[(size_t)(l - rows)]; };
    for (int64_t r = 0; r < rows; ++r) {
        const int64_t beg = pl.lip[r], end = pl.lip[r + 1];
        const bool whole = whole_max > 0 && end - beg <= whole_max;
        for (int b = 1; b < B; ++b) {
            if (whole) { sp[b - 1][r] = end; continue; }
            const int64_t bound = ((int64_t)b * pl.n + B - 1) / B;
            int64_t lo = beg, hi = end;
            while (lo < hi) {
                const int64_t mid = lo + (hi - lo) / 2;
                if (glob(pl.lix[mid]) < bound) lo = mid + 1; else hi = mid;
            }
            sp[b - 1][r] = lo;
        }
    }
    auto bound_at = [&](int b, int64_t r) { return b == 0 ? pl.lip[r] : b == B ? pl.lip[r + 1] : sp[b - 1][r]; };
    const int64_t heavy_t = pl.auto_heavy ? auto_heavy(pl.b1 - pl.b0, C * B) : pl.heavy_threshold;
    K.views.assign(C, std::vector<SrgHaloView>(B));
    for (int c = 0; c < C; ++c) {
        const std::vector<int32_t>& rows_c = pl.views[c].order;
        std::vector<int32_t> cut;
        for (int32_t r : rows_c)
            if (!(whole_max > 0 && pl.lip[r + 1] - pl.lip[r] <= whole_max)) cut.push_back(r);
        for (int b = 0; b < B; ++b) {
            SrgHaloView& V = K.views[c][b];
            V.order = b == 0 ? rows_c : cut;
            std::vector<int64_t> len(V.order.size());
            for (size_t i = 0; i < V.order.size(); ++i) len[i] = bound_at(b + 1, V.order[i]) - bound_at(b, V.order[i]);
            std::vector<int32_t> idx(V.order.size());
            for (size_t i = 0; i < idx.size(); ++i) idx[i] = (int32_t)i;
            std::stable_sort(idx.begin(), idx.end(), [&](int32_t a, int32_t b2) { return len[a] > len[b2]; });
            std::vector<int32_t> o(idx.size());
            for (size_t i = 0; i < idx.size(); ++i) o[i] = V.order[idx[i]];
            V.order.swap(o);
            V.n = (int64_t)V.order.size();
            for (int64_t l : len) {
                V.n_heavy += (heavy_t >= 0 && l > heavy_t) ? 1 : 0;
                V.n_heavy_narrow += l > kNarrowHeavy ? 1 : 0;
            }
            if (!pl.auto_heavy) V.n_heavy_narrow = V.n_heavy;
        }
    }
    // device arrays
    K.B = B;
    K.splits.assign((size_t)B - 1, nullptr);
    K.bounds.assign((size_t)B + 1, nullptr);
    K.bounds[0] = S->lip;
    K.bounds[B] = S->lip + 1;
    for (int b = 1; b < B; ++b) {
        if (rows == 0) continue;
        if (hipMalloc((void**)&K.splits[b - 1], (size_t)rows * sizeof(int64_t)) != hipSuccess)
            return hfail(SRG_ERR_ALLOC, "column block split points (%lld rows)", (long long)rows);
        SRG_HALO_HIP(hipMemcpy(K.splits[b - 1], sp[b - 1].data(), (size_t)rows * sizeof(int64_t), hipMemcpyHostToDevice));
        K.bounds[b] = K.splits[b - 1];
    }
    K.orders.assign(C, std::vector<int32_t*>(B, nullptr));
    for (int c = 0; c < C; ++c)
        for (int b = 0; b < B; ++b) {
            std::vector<int32_t>& o = K.views[c][b].order;
            if (!o.empty()) {
                if (hipMalloc((void**)&K.orders[c][b], o.size() * sizeof(int32_t)) != hipSuccess)
                    return hfail(SRG_ERR_ALLOC, "column block schedule (%zu rows)", o.size());
                SRG_HALO_HIP(hipMemcpy(K.orders[c][b], o.data(), o.size() * sizeof(int32_t), hipMemcpyHostToDevice));
            }
            std::vector<int32_t>().swap(o);
        }
    return SRG_OK;
}

}  // namespace

int srg_halo_col_blocks(int64_t nloc, int d)
{
    const int64_t panel = nloc * (int64_t)d * 4;
    return (d >= 256 && panel >= (8ll << 30)) ? 8 : 1;
}

extern "C" {

int srg_halo_plan_build(const int64_t* indptr, const int32_t* indices, int64_t n, int32_t nranks, int32_t rank,
                        int32_t chunks, int64_t hub_threshold, int64_t heavy_threshold, int32_t ghost_max_degree,
                        double link_bps, srg_halo_plan** out)
{
    if (!out) return hfail(SRG_ERR_INVALID, "null output handle");
    *out = nullptr;
    if (!indptr || (n > 0 && !indices)) return hfail(SRG_ERR_INVALID, "null indptr / indices");
    if (n < 0 || n > INT32_MAX - 1) return hfail(SRG_ERR_INVALID, "n=%lld out of range", (long long)n);
    if (nranks < 1 || rank < 0 || rank >= nranks) return hfail(SRG_ERR_INVALID, "rank %d of %d", rank, nranks);
    if (chunks < 1 || chunks > 250) return hfail(SRG_ERR_INVALID, "chunks=%d not in [1, 250]", chunks);
    const bool auto_ghost = ghost_max_degree == SRG_HALO_AUTO;
    if (ghost_max_degree < 0 && !auto_ghost)
        return hfail(SRG_ERR_INVALID, "ghost_max_degree=%d < 0 (SRG_HALO_AUTO: the cost model)", ghost_max_degree);
    if (hub_threshold < SRG_HALO_NONE || heavy_threshold < SRG_HALO_AUTO)
        return hfail(SRG_ERR_INVALID, "thresholds: hub %lld, heavy %lld", (long long)hub_threshold, (long long)heavy_threshold);
    if (indptr[0] != 0) return hfail(SRG_ERR_INVALID, "indptr[0] = %lld != 0", (long long)indptr[0]);
    {
        // the checks in parallel pieces; the first violation (lowest position) is reported
        std::vector<int64_t> bad_row((size_t)plan_threads() + 1, INT64_MAX);
        std::atomic<int> slot{0};
        parallel_ranges(n, [&](int64_t lo, int64_t hi) {
            int64_t b = INT64_MAX;
            for (int64_t r = lo; r < hi && b == INT64_MAX; ++r)
                if (indptr[r + 1] < indptr[r]) b = r;
            bad_row[(size_t)slot++] = b;
        });
        const int64_t b = *std::min_element(bad_row.begin(), bad_row.end());
        if (b != INT64_MAX) return hfail(SRG_ERR_INVALID, "indptr decreases at row %lld", (long long)b);
    }
    const int64_t nnz = indptr[n];
    {
        std::vector<int64_t> bad_e((size_t)plan_threads() + 1, INT64_MAX);
        std::atomic<int> slot{0};
        parallel_ranges(nnz, [&](int64_t lo, int64_t hi) {
            int64_t b = INT64_MAX;
            for (int64_t e = lo; e < hi && b == INT64_MAX; ++e)
                if (indices[e] < 0 || indices[e] >= n) b = e;
            bad_e[(size_t)slot++] = b;
        });
        const int64_t e = *std::min_element(bad_e.begin(), bad_e.end());
        if (e != INT64_MAX)
            return hfail(SRG_ERR_INVALID, "column id %d at entry %lld outside [0, %lld)", indices[e], (long long)e, (long long)n);
    }

    srg_halo_plan* P_ = new (std::nothrow) srg_halo_plan();
    if (!P_) return hfail(SRG_ERR_ALLOC, "out of host memory");
    srg_halo_plan& pl = *P_;
    const int P = nranks, p = rank, C = chunks, G = C + 1;
    pl.P = P; pl.p = p; pl.C = C; pl.n = n; pl.nnz_total = nnz;
    const int scan_cap = auto_ghost ? kGhostScanMax : ghost_max_degree;   // ghost candidates scanned up to
    pl.starts = balanced(indptr, n, P, 0);
    const std::vector<int64_t>& st = pl.starts;
    auto deg = [&](int64_t r) { return indptr[r + 1] - indptr[r]; };

    // owner rank and group of every row
    std::vector<int32_t> owner(n);
    std::vector<uint8_t> grp(n);
    pl.hub_thresholds.assign(P, 0);
    for (int q = 0; q < P; ++q) {
        const int64_t s0 = st[q], s1 = st[q + 1];
        const int64_t nnz_q = indptr[s1] - indptr[s0];
        const int64_t thr = hub_threshold == SRG_HALO_AUTO ? auto_hub(nnz_q, C)
                          : hub_threshold == SRG_HALO_NONE ? INT64_MAX : hub_threshold;
        pl.hub_thresholds[q] = thr;
        const std::vector<int64_t> cb = balanced(indptr + s0, s1 - s0, C, indptr[s0]);
        for (int c = 0; c < C; ++c)
            for (int64_t r = s0 + cb[c]; r < s0 + cb[c + 1]; ++r) {
                owner[r] = q;
                grp[r] = (uint8_t)(deg(r) > thr ? C : c);
            }
        if (q == p) pl.chunk_ranges = cb;
    }

    // every rank's halo, sorted by (group, owner, id), its ghost-eligible rows (one thread per rank),
    // and for the automatic cap each rank's modelled SpMM entries and busiest link per candidate cap
    std::vector<std::vector<int32_t>> halos(P);
    std::vector<std::vector<uint8_t>> ghost(P);
    std::vector<std::vector<int64_t>> model_nnz(P, std::vector<int64_t>(kNumGhostCaps, 0));
    std::vector<std::vector<int64_t>> model_link(P, std::vector<int64_t>(kNumGhostCaps, 0));
    auto halo_of = [&](int q) {
        const int64_t s0 = st[q], s1 = st[q + 1];
        std::vector<uint64_t> bits((size_t)(n + 63) / 64, 0);
        for (int64_t e = indptr[s0]; e < indptr[s1]; ++e) {
            const int32_t c = indices[e];
            if (c < s0 || c >= s1) bits[c >> 6] |= 1ull << (c & 63);
        }
        // counting sort by (group, owner) of the ids in ascending order: (group, owner, id)
        std::vector<int64_t> cnt((size_t)G * P + 1, 0);
        for (size_t w = 0; w < bits.size(); ++w)
            for (uint64_t b = bits[w]; b; b &= b - 1) {
                const int64_t c = (int64_t)(w * 64 + __builtin_ctzll(b));
                ++cnt[(size_t)grp[c] * P + owner[c] + 1];
            }
        for (size_t k = 1; k < cnt.size(); ++k) cnt[k] += cnt[k - 1];
        std::vector<int32_t>& h = halos[q];
        h.assign((size_t)cnt.back(), 0);
        for (size_t w = 0; w < bits.size(); ++w)
            for (uint64_t b = bits[w]; b; b &= b - 1) {
                const int32_t c = (int32_t)(w * 64 + __builtin_ctzll(b));
                h[(size_t)cnt[(size_t)grp[c] * P + owner[c]]++] = c;
            }
        // ghosts: degree <= cap and every column among q's own rows or halo rows
        std::vector<uint8_t>& g = ghost[q];
        g.assign(h.size(), 0);
        if (scan_cap > 0)
            for (size_t j = 0; j < h.size(); ++j) {
                const int32_t r = h[j];
                if (deg(r) > scan_cap) continue;
                bool ok = true;
                for (int64_t e = indptr[r]; e < indptr[r + 1] && ok; ++e) {
                    const int32_t c = indices[e];
                    ok = (c >= s0 && c < s1) || ((bits[c >> 6] >> (c & 63)) & 1ull);
                }
                g[j] = ok ? 1 : 0;
            }
        if (auto_ghost) {
            // per cap: q's SpMM entries (own + ghost rows) and its busiest inbound link (rows received
            // from one owner) -- dist.ghost_plan's model
            std::vector<int64_t> recv((size_t)kNumGhostCaps * P, 0);
            std::vector<int64_t> gnnz(kNumGhostCaps, 0);
            for (size_t j = 0; j < h.size(); ++j) {
                const int64_t dr = deg(h[j]);
                for (int k = 0; k < kNumGhostCaps; ++k) {
                    if (g[j] && dr <= kGhostCaps[k]) gnnz[k] += dr;
                    else ++recv[(size_t)k * P + owner[h[j]]];
                }
            }
            for (int k = 0; k < kNumGhostCaps; ++k) {
                model_nnz[q][k] = indptr[s1] - indptr[s0] + gnnz[k];
                model_link[q][k] = *std::max_element(recv.begin() + (size_t)k * P, recv.begin() + (size_t)(k + 1) * P);
            }
        }
    };
    {
        const int nt = (int)std::max(1u, std::min<unsigned>(std::thread::hardware_concurrency(), 16u));
        for (int q0 = 0; q0 < P; q0 += nt) {
            std::vector<std::thread> th;
            for (int q = q0; q < std::min(P, q0 + nt); ++q) th.emplace_back(halo_of, q);
            for (auto& t : th) t.join();
        }
    }

    // the ghost cap: given, or the candidate with the least modelled hop (ties: the smaller cap)
    int cap = ghost_max_degree;
    if (auto_ghost) {
        const double link = link_bps > 0 ? link_bps : kGhostLinkBps;
        double best_t = 0;
        for (int k = 0; k < kNumGhostCaps; ++k) {
            double worst = 0.0;
            for (int q = 0; q < P; ++q)
                worst = std::max(worst, std::max((double)model_nnz[q][k] / kGhostGatherBps, (double)model_link[q][k] / link));
            if (k == 0 || worst < best_t) { best_t = worst; cap = kGhostCaps[k]; }
        }
        for (int q = 0; q < P; ++q)
            for (size_t j = 0; j < halos[q].size(); ++j)
                if (ghost[q][j] && deg(halos[q][j]) > cap) ghost[q][j] = 0;
    }
    pl.ghost_max_degree = cap;

    const int64_t r0 = st[p], r1 = st[p + 1];
    pl.r0 = r0; pl.r1 = r1; pl.rows = r1 - r0;
    pl.b0 = indptr[r0]; pl.b1 = indptr[r1];
    // received rows (halo order) and ghosts (by owner, id)
    std::vector<int32_t> need, gh;
    for (size_t j = 0; j < halos[p].size(); ++j) (ghost[p][j] ? gh : need).push_back(halos[p][j]);
    std::stable_sort(gh.begin(), gh.end(), [&](int32_t a, int32_t b) {
        return owner[a] != owner[b] ? owner[a] < owner[b] : a < b; });
    pl.n_recv = (int64_t)need.size();
    pl.n_ghost = (int64_t)gh.size();
    pl.halo = pl.n_recv + pl.n_ghost;
    pl.recv_counts.assign(G, std::vector<int64_t>(P, 0));
    for (int32_t c : need) ++pl.recv_counts[grp[c]][owner[c]];
    pl.ghost_recv_counts.assign(P, 0);
    for (int32_t c : gh) ++pl.ghost_recv_counts[owner[c]];
    pl.group_offsets.assign(G, 0);
    for (int g = 1; g < G; ++g) {
        int64_t s = 0;
        for (int q = 0; q < P; ++q) s += pl.recv_counts[g - 1][q];
        pl.group_offsets[g] = pl.group_offsets[g - 1] + s;
    }
    // sends: for every peer q, my rows q receives, per group in q's receive order, and my rows q
    // computes as ghosts, by id
    pl.send_counts.assign(G, std::vector<int64_t>(P, 0));
    pl.send_cat.assign(G, {});
    pl.ghost_send_counts.assign(P, 0);
    for (int q = 0; q < P; ++q) {
        if (q == p) continue;
        std::vector<int64_t> gs;
        for (size_t j = 0; j < halos[q].size(); ++j) {
            const int32_t c = halos[q][j];
            if (owner[c] != p) continue;
            if (ghost[q][j]) { gs.push_back(c - r0); continue; }
            pl.send_cat[grp[c]].push_back(c - r0);
            ++pl.send_counts[grp[c]][q];
        }
        std::sort(gs.begin(), gs.end());
        pl.ghost_send_counts[q] = (int64_t)gs.size();
        pl.ghost_send_cat.insert(pl.ghost_send_cat.end(), gs.begin(), gs.end());
    }
    halos.clear();
    ghost.clear();

    // local CSR over [own | received | ghosts], columns remapped into the panel
    std::vector<int32_t> g2l(n, -1);
    for (int64_t i = 0; i < pl.rows; ++i) g2l[r0 + i] = (int32_t)i;
    for (int64_t j = 0; j < pl.n_recv; ++j) g2l[need[j]] = (int32_t)(pl.rows + j);
    for (int64_t j = 0; j < pl.n_ghost; ++j) g2l[gh[j]] = (int32_t)(pl.rows + pl.n_recv + j);
    const int64_t nloc = pl.rows + pl.halo;
    pl.lip.assign(nloc + 1, 0);
    for (int64_t i = 0; i < pl.rows; ++i) pl.lip[i + 1] = pl.lip[i] + deg(r0 + i);
    for (int64_t j = 0; j < pl.n_recv; ++j) pl.lip[pl.rows + j + 1] = pl.lip[pl.rows + j];
    for (int64_t j = 0; j < pl.n_ghost; ++j) pl.lip[pl.rows + pl.n_recv + j + 1] = pl.lip[pl.rows + pl.n_recv + j] + deg(gh[j]);
    pl.lix.resize((size_t)pl.lip[nloc]);
    parallel_ranges(pl.b1 - pl.b0, [&](int64_t lo, int64_t hi) {
        for (int64_t e = lo; e < hi; ++e) pl.lix[(size_t)e] = g2l[indices[pl.b0 + e]];
    });
    int64_t w = pl.b1 - pl.b0;
    for (int32_t r : gh)
        for (int64_t e = indptr[r]; e < indptr[r + 1]; ++e) {
            pl.ghost_pos.push_back(e);
            pl.lix[w++] = g2l[indices[e]];
        }
    {
        std::atomic<bool> miss{false};
        parallel_ranges((int64_t)pl.lix.size(), [&](int64_t lo, int64_t hi) {
            for (int64_t e = lo; e < hi; ++e)
                if (pl.lix[(size_t)e] < 0) { miss = true; break; }
        });
        if (miss) {
            delete P_;
            return hfail(SRG_ERR_INVALID, "halo layout misses a referenced column");
        }
    }
    pl.halo_ids.reserve(pl.halo);
    pl.halo_ids.insert(pl.halo_ids.end(), need.begin(), need.end());
    pl.halo_ids.insert(pl.halo_ids.end(), gh.begin(), gh.end());

    // schedules: the C chunks and the hub group over the own rows, then the ghost rows
    std::vector<int64_t> ldeg(nloc);
    for (int64_t i = 0; i < nloc; ++i) ldeg[i] = pl.lip[i + 1] - pl.lip[i];
    const bool auto_h = heavy_threshold == SRG_HALO_AUTO;
    const int64_t heavy_t = auto_h ? std::max<int64_t>(kHaloHeavyMin, auto_heavy(pl.b1 - pl.b0, C)) : heavy_threshold;
    pl.heavy_threshold = heavy_t;
    pl.auto_heavy = auto_h;
    pl.views.assign(G + 1, {});
    for (int64_t i = 0; i < pl.rows; ++i) pl.views[grp[r0 + i]].order.push_back((int32_t)i);
    for (int64_t j = 0; j < pl.n_ghost; ++j) pl.views[G].order.push_back((int32_t)(pl.rows + pl.n_recv + j));
    for (int v = 0; v <= G; ++v) {
        SrgHaloView& V = pl.views[v];
        sort_by_degree(V.order, ldeg);
        V.n = (int64_t)V.order.size();
        if (v == C) {                  // the hub group: every row a hub row
            V.n_hub = V.n;
            continue;
        }
        for (int32_t r : V.order) {
            V.n_heavy += ldeg[r] > heavy_t ? 1 : 0;
            V.n_heavy_narrow += ldeg[r] > kNarrowHeavy ? 1 : 0;
        }
        if (!auto_h) V.n_heavy_narrow = V.n_heavy;
    }
    *out = P_;
    srg_clear_error();
    return SRG_OK;
}

int srg_halo_plan_destroy(srg_halo_plan* plan)
{
    delete plan;
    return SRG_OK;
}

int srg_halo_plan_info(const srg_halo_plan* plan, srg_halo_info* info)
{
    if (!plan || !info) return hfail(SRG_ERR_INVALID, "null argument");
    const srg_halo_plan& pl = *plan;
    info->row0 = pl.r0;
    info->n_rows = pl.rows;
    info->n_recv = pl.n_recv;
    info->n_ghost = pl.n_ghost;
    info->halo = pl.halo;
    info->nnz_local = (int64_t)pl.lix.size();
    info->n_groups = pl.C + 1;
    info->hub_rows = pl.views[pl.C].n;
    int64_t s = 0;
    for (auto& v : pl.send_cat) s += (int64_t)v.size();
    info->send_rows = s;
    info->ghost_max_degree = pl.ghost_max_degree;
    info->chunks = pl.C;
    info->nranks = pl.P;
    info->rank = pl.p;
    return SRG_OK;
}

int srg_halo_plan_array(const srg_halo_plan* plan, int32_t what, int32_t index, const void** data, int64_t* count)
{
    if (!plan || !data || !count) return hfail(SRG_ERR_INVALID, "null argument");
    const srg_halo_plan& pl = *plan;
    const int G = pl.C + 1;
    auto put = [&](const auto& v) { *data = v.data(); *count = (int64_t)v.size(); return SRG_OK; };
    static thread_local int64_t meta[4];
    switch (what) {
    case SRG_HALO_STARTS: return put(pl.starts);
    case SRG_HALO_LOCAL_INDPTR: return put(pl.lip);
    case SRG_HALO_LOCAL_INDICES: return put(pl.lix);
    case SRG_HALO_GHOST_POSITIONS: return put(pl.ghost_pos);
    case SRG_HALO_HALO_IDS: return put(pl.halo_ids);
    case SRG_HALO_GROUP_OFFSETS: return put(pl.group_offsets);
    case SRG_HALO_GHOST_SEND: return put(pl.ghost_send_cat);
    case SRG_HALO_GHOST_SEND_COUNTS: return put(pl.ghost_send_counts);
    case SRG_HALO_GHOST_RECV_COUNTS: return put(pl.ghost_recv_counts);
    case SRG_HALO_CHUNK_RANGES: return put(pl.chunk_ranges);
    case SRG_HALO_HUB_THRESHOLDS: return put(pl.hub_thresholds);
    default: break;
    }
    if (what == SRG_HALO_VIEW_ORDER || what == SRG_HALO_VIEW_META) {
        if (index < 0 || index > G) return hfail(SRG_ERR_INVALID, "view %d of %d", index, G + 1);
        const SrgHaloView& V = pl.views[index];
        if (what == SRG_HALO_VIEW_ORDER) return put(V.order);
        meta[0] = V.n; meta[1] = V.n_hub; meta[2] = V.n_heavy; meta[3] = V.n_heavy_narrow;
        *data = meta;
        *count = 4;
        return SRG_OK;
    }
    if (index < 0 || index >= G) return hfail(SRG_ERR_INVALID, "group %d of %d", index, G);
    switch (what) {
    case SRG_HALO_SEND_ROWS: return put(pl.send_cat[index]);
    case SRG_HALO_SEND_COUNTS: return put(pl.send_counts[index]);
    case SRG_HALO_RECV_COUNTS: return put(pl.recv_counts[index]);
    default: return hfail(SRG_ERR_INVALID, "unknown plan array %d", what);
    }
}

int srg_halo_share_create(const srg_halo_plan* plan, const float* values, int device, int32_t d_max,
                          srg_halo_share** out)
{
    if (!out) return hfail(SRG_ERR_INVALID, "null output handle");
    *out = nullptr;
    if (!plan || (plan->nnz_total > 0 && !values)) return hfail(SRG_ERR_INVALID, "null plan / values");
    if (d_max < 1) return hfail(SRG_ERR_INVALID, "d_max=%d < 1", d_max);
    const srg_halo_plan& pl = *plan;
    int prev = -1;
    if (hipGetDevice(&prev) != hipSuccess) return hfail(SRG_ERR_HIP, "no HIP device");
    SRG_HALO_HIP(hipSetDevice(device));
    struct Restore { int d; ~Restore() { (void)hipSetDevice(d); } } restore{prev};
    srg_halo_share* S = new (std::nothrow) srg_halo_share();
    if (!S) return hfail(SRG_ERR_ALLOC, "out of host memory");
    S->device = device;
    S->plan = plan;
    S->d_cap = d_max;
    auto fail_free = [&](int rc) { srg_halo_share_destroy(S); return rc; };
    auto upload = [&](void** dst, const void* src, size_t bytes) -> int {
        if (bytes == 0) return SRG_OK;
        if (hipMalloc(dst, bytes) != hipSuccess) return hfail(SRG_ERR_ALLOC, "hipMalloc(%zu) failed", bytes);
        if (hipMemcpy(*dst, src, bytes, hipMemcpyHostToDevice) != hipSuccess)
            return hfail(SRG_ERR_HIP, "hipMemcpy of %zu bytes failed", bytes);
        return SRG_OK;
    };
    // the local values: the own rows' entries, then the ghost rows' (host gather of the global array)
    const int64_t nl = (int64_t)pl.lix.size();
    std::vector<float> lv((size_t)nl);
    if (pl.b1 > pl.b0) memcpy(lv.data(), values + pl.b0, (size_t)(pl.b1 - pl.b0) * sizeof(float));
    for (size_t j = 0; j < pl.ghost_pos.size(); ++j) lv[(size_t)(pl.b1 - pl.b0) + j] = values[pl.ghost_pos[j]];
    int rc = upload((void**)&S->lip, pl.lip.data(), pl.lip.size() * sizeof(int64_t));
    if (!rc) rc = upload((void**)&S->lix, pl.lix.data(), pl.lix.size() * sizeof(int32_t));
    if (!rc) rc = upload((void**)&S->lvv, lv.data(), lv.size() * sizeof(float));
    if (rc) return fail_free(rc);
    S->orders.assign(pl.views.size(), nullptr);
    for (size_t v = 0; v < pl.views.size() && !rc; ++v)
        rc = upload((void**)&S->orders[v], pl.views[v].order.data(), pl.views[v].order.size() * sizeof(int32_t));
    const int G = pl.C + 1;
    S->send_idx.assign(G + 1, nullptr);
    S->send_off.assign(G + 2, 0);
    for (int g = 0; g <= G && !rc; ++g) {
        const std::vector<int64_t>& v = g < G ? pl.send_cat[g] : pl.ghost_send_cat;
        rc = upload((void**)&S->send_idx[g], v.data(), v.size() * sizeof(int64_t));
        S->send_off[g + 1] = S->send_off[g] + (int64_t)v.size();
    }
    if (rc) return fail_free(rc);
    if (S->send_off.back() > 0 &&
        hipMalloc((void**)&S->sendbuf, (size_t)S->send_off.back() * (size_t)d_max * sizeof(float)) != hipSuccess)
        return fail_free(hfail(SRG_ERR_ALLOC, "send buffer of %lld rows x %d", (long long)S->send_off.back(), d_max));
    const int B = srg_halo_col_blocks(pl.rows + pl.halo, d_max);
    if (B > 1 && (rc = build_blocks(S, B))) return fail_free(rc);
    S->packed.assign(G + 1, nullptr);
    for (auto& e : S->packed)
        if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess)
            return fail_free(hfail(SRG_ERR_HIP, "hipEventCreate failed"));
    if (hipEventCreateWithFlags(&S->comm_done, hipEventDisableTiming) != hipSuccess ||
        hipStreamCreateWithFlags(&S->comm_stream, hipStreamNonBlocking) != hipSuccess)
        return fail_free(hfail(SRG_ERR_HIP, "comm stream / event creation failed"));
    *out = S;
    srg_clear_error();
    return SRG_OK;
}

int srg_halo_share_destroy(srg_halo_share* S)
{
    if (!S) return SRG_OK;
    int prev = -1;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(S->device);
    if (S->comm_stream) (void)hipStreamSynchronize(S->comm_stream);
    (void)hipFree(S->lip);
    (void)hipFree(S->lix);
    (void)hipFree(S->lvv);
    for (auto* o : S->orders) (void)hipFree(o);
    free_blocks(S->blocks);
    for (auto* s : S->send_idx) (void)hipFree(s);
    (void)hipFree(S->sendbuf);
    for (auto e : S->packed) if (e) (void)hipEventDestroy(e);
    if (S->comm_done) (void)hipEventDestroy(S->comm_done);
    if (S->comm_stream) (void)hipStreamDestroy(S->comm_stream);
    if (prev >= 0) (void)hipSetDevice(prev);
    delete S;
    return SRG_OK;
}

int srg_halo_share_col_blocks(srg_halo_share* S, int32_t n_blocks)
{
    if (!S || !S->plan) return hfail(SRG_ERR_INVALID, "null share");
    if (n_blocks != SRG_HALO_AUTO && (n_blocks < 1 || n_blocks > 64))
        return hfail(SRG_ERR_INVALID, "n_blocks=%d not in [1, 64] nor SRG_HALO_AUTO", n_blocks);
    int prev = -1;
    if (hipGetDevice(&prev) != hipSuccess) return hfail(SRG_ERR_HIP, "no HIP device");
    SRG_HALO_HIP(hipSetDevice(S->device));
    struct Restore { int d; ~Restore() { (void)hipSetDevice(d); } } restore{prev};
    SRG_HALO_HIP(hipDeviceSynchronize());          // no launch of this share may still read the old arrays
    free_blocks(S->blocks);
    const srg_halo_plan& pl = *S->plan;
    const int B = n_blocks == SRG_HALO_AUTO ? srg_halo_col_blocks(pl.rows + pl.halo, (int)S->d_cap) : n_blocks;
    int rc = B > 1 ? build_blocks(S, B) : SRG_OK;
    if (rc) {
        free_blocks(S->blocks);
        return rc;
    }
    S->blocks.forced = n_blocks != SRG_HALO_AUTO;
    srg_clear_error();
    return SRG_OK;
}

int srg_halo_fill_x_halo(const srg_halo_share* S, const float* X, int64_t ldx, float* panel0, int64_t ld, int32_t d,
                         void* stream)
{
    if (!S || !X || !panel0) return hfail(SRG_ERR_INVALID, "null argument");
    const srg_halo_plan& pl = *S->plan;
    if (ld < d || ldx < d) return hfail(SRG_ERR_INVALID, "leading dimensions < d");
    // own rows, then the halo rows gathered by global id (the ids live on the host: one upload)
    int64_t* ids = nullptr;
    int prev = -1;
    if (hipGetDevice(&prev) != hipSuccess) return hfail(SRG_ERR_HIP, "no HIP device");
    SRG_HALO_HIP(hipSetDevice(S->device));
    struct Restore { int d; ~Restore() { (void)hipSetDevice(d); } } restore{prev};
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (pl.rows)
        SRG_HALO_HIP(hipMemcpy2DAsync(panel0, (size_t)ld * 4, X + pl.r0 * ldx, (size_t)ldx * 4, (size_t)d * 4,
                                      (size_t)pl.rows, hipMemcpyDeviceToDevice, s));
    if (pl.halo == 0) return SRG_OK;
    SRG_HALO_HIP(hipMallocAsync((void**)&ids, (size_t)pl.halo * sizeof(int64_t), s));
    SRG_HALO_HIP(hipMemcpyAsync(ids, pl.halo_ids.data(), (size_t)pl.halo * sizeof(int64_t), hipMemcpyHostToDevice, s));
    int rc = srg_gather_rows_f32(X, ldx, pl.n, ids, pl.halo, panel0 + pl.rows * ld, ld, d, stream);
    SRG_HALO_HIP(hipFreeAsync(ids, s));
    SRG_HALO_HIP(hipStreamSynchronize(s));      // the host id array is pageable: keep it alive
    return rc;
}

}  // extern "C"
