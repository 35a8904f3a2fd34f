/*
 * examples/halo_loopback.c -- a plain C host of libsrgnn_hip.so (no Python, no torch): the K-hop
 * propagation of a synthetic normalised graph on one GPU (srg_propagate_khop_f32), then the same K
 * hops over the halo-exchange partition of P ranks (srg_halo_plan_build / srg_halo_share_create /
 * srg_halo_propagate_f32) through the loopback communicator, and a bitwise comparison of every rank's
 * own rows of every hop.  Exit status 0 = bitwise equal.  Shows the C-ABI of include/srgnn_hip.h
 * compiles as C and drives the multi-rank path end to end.
 *
 *   examples/halo_loopback [P] [n] [d] [K]        (defaults 4 20000 64 4)
 */
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "srgnn_hip.h"

#define CHECK(x)                                                                             \
    do {                                                                                     \
        int rc_ = (x);                                                                       \
        if (rc_) {                                                                           \
            fprintf(stderr, "%s:%d %s -> %d: %s\n", __FILE__, __LINE__, #x, rc_, srg_last_error()); \
            return 2;                                                                        \
        }                                                                                    \
    } while (0)
#define HCHECK(x)                                                                            \
    do {                                                                                     \
        hipError_t e_ = (x);                                                                 \
        if (e_ != hipSuccess) {                                                              \
            fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            return 2;                                                                        \
        }                                                                                    \
    } while (0)

static uint64_t rng = 0x9e3779b97f4a7c15ull;
static uint64_t next(void) { rng ^= rng << 13; rng ^= rng >> 7; rng ^= rng << 17; return rng; }

static int cmp64(const void* a, const void* b)
{
    int64_t x = *(const int64_t*)a, y = *(const int64_t*)b;
    return x < y ? -1 : x > y;
}

int main(int argc, char** argv)
{
    const int P = argc > 1 ? atoi(argv[1]) : 4;
    const int64_t n = argc > 2 ? atoll(argv[2]) : 20000;
    const int d = argc > 3 ? atoi(argv[3]) : 64;
    const int K = argc > 4 ? atoi(argv[4]) : 4;
    /* a symmetric graph with a power-law-ish degree skew (edge endpoints drawn from a squared
     * uniform), self-loops, duplicates removed; values 1/sqrt(deg_i deg_j) rounded to fp32 */
    const int64_t m = 10 * n;
    int64_t* key = malloc(sizeof(int64_t) * (2 * m + n));
    int64_t e = 0;
    for (int64_t i = 0; i < m; ++i) {
        double a = (double)(next() % 1000003) / 1000003.0, b = (double)(next() % 1000003) / 1000003.0;
        int64_t u = (int64_t)(a * a * n), v = (int64_t)(b * n);
        if (u == v) continue;
        key[e++] = u * n + v;
        key[e++] = v * n + u;
    }
    for (int64_t i = 0; i < n; ++i) key[e++] = i * n + i;
    qsort(key, e, sizeof(int64_t), cmp64);
    int64_t nnz = 0;
    for (int64_t i = 0; i < e; ++i)
        if (i == 0 || key[i] != key[i - 1]) key[nnz++] = key[i];
    int64_t* ip = calloc(n + 1, sizeof(int64_t));
    int32_t* ix = malloc(sizeof(int32_t) * nnz);
    float* val = malloc(sizeof(float) * nnz);
    for (int64_t i = 0; i < nnz; ++i) { ++ip[key[i] / n + 1]; ix[i] = (int32_t)(key[i] % n); }
    for (int64_t r = 0; r < n; ++r) ip[r + 1] += ip[r];
    for (int64_t r = 0; r < n; ++r)
        for (int64_t j = ip[r]; j < ip[r + 1]; ++j) {
            double dr = (double)(ip[r + 1] - ip[r]), dc = (double)(ip[ix[j] + 1] - ip[ix[j]]);
            val[j] = (float)(1.0 / __builtin_sqrt(dr * dc));
        }
    float* X = malloc(sizeof(float) * n * d);
    for (int64_t i = 0; i < n * d; ++i) X[i] = (float)((double)(next() % 2000001) / 1000000.0 - 1.0);

    /* one GPU: K hops, all panels */
    int64_t *d_ip; int32_t* d_ix; float *d_v, *d_X;
    HCHECK(hipMalloc((void**)&d_ip, sizeof(int64_t) * (n + 1)));
    HCHECK(hipMalloc((void**)&d_ix, sizeof(int32_t) * nnz));
    HCHECK(hipMalloc((void**)&d_v, sizeof(float) * nnz));
    HCHECK(hipMemcpy(d_ip, ip, sizeof(int64_t) * (n + 1), hipMemcpyHostToDevice));
    HCHECK(hipMemcpy(d_ix, ix, sizeof(int32_t) * nnz, hipMemcpyHostToDevice));
    HCHECK(hipMemcpy(d_v, val, sizeof(float) * nnz, hipMemcpyHostToDevice));
    CHECK(srg_csr_validate(d_ip, d_ix, n, nnz, n, NULL));
    float** one = malloc(sizeof(float*) * (K + 1));
    for (int k = 0; k <= K; ++k) HCHECK(hipMalloc((void**)&one[k], sizeof(float) * n * d));
    HCHECK(hipMemcpy(one[0], X, sizeof(float) * n * d, hipMemcpyHostToDevice));
    d_X = one[0];
    CHECK(srg_propagate_khop_f32(d_ip, d_ix, d_v, n, NULL, 0, 0, one, d, d, K, 0u, NULL));

    /* P ranks over the halo partition, one process, one GPU: loopback exchange */
    srg_comm* comm;
    CHECK(srg_comm_init_loopback(P, 0, &comm));
    srg_halo_plan** plan = malloc(sizeof(void*) * P);
    srg_halo_share** share = malloc(sizeof(void*) * P);
    float*** panels = malloc(sizeof(float**) * P);
    void** streams = malloc(sizeof(void*) * P);
    srg_halo_info* info = malloc(sizeof(srg_halo_info) * P);
    for (int p = 0; p < P; ++p) {
        CHECK(srg_halo_plan_build(ip, ix, n, P, p, 3, SRG_HALO_AUTO, SRG_HALO_AUTO, /*ghost_max_degree=*/4, 0.0, &plan[p]));
        CHECK(srg_halo_plan_info(plan[p], &info[p]));
        CHECK(srg_halo_share_create(plan[p], val, 0, d, &share[p]));
        panels[p] = malloc(sizeof(float*) * (K + 1));
        const int64_t rows = info[p].n_rows + info[p].halo;
        for (int k = 0; k <= K; ++k) HCHECK(hipMalloc((void**)&panels[p][k], sizeof(float) * (rows > 0 ? rows : 1) * d));
        HCHECK(hipStreamCreate((hipStream_t*)&streams[p]));
        /* even ranks fill hop 0's halo from the whole X, odd ranks let the exchange bring it: both are
         * tested, but one call takes one mode, so here every rank fills it */
        CHECK(srg_halo_fill_x_halo(share[p], d_X, d, panels[p][0], d, d, streams[p]));
    }
    CHECK(srg_halo_propagate_f32(comm, share, P, (float* const* const*)panels, d, d, K, SRG_HALO_X_HALO_FILLED, streams));
    HCHECK(hipDeviceSynchronize());

    /* every rank's own rows of every hop == the one-GPU hop, bit for bit */
    int bad = 0;
    float* a = malloc(sizeof(float) * n * d);
    float* b = malloc(sizeof(float) * n * d);
    for (int k = 1; k <= K; ++k) {
        HCHECK(hipMemcpy(a, one[k], sizeof(float) * n * d, hipMemcpyDeviceToHost));
        for (int p = 0; p < P; ++p) {
            const int64_t r0 = info[p].row0, rows = info[p].n_rows;
            if (!rows) continue;
            HCHECK(hipMemcpy(b, panels[p][k], sizeof(float) * rows * d, hipMemcpyDeviceToHost));
            if (memcmp(a + r0 * d, b, sizeof(float) * rows * d)) {
                fprintf(stderr, "hop %d rank %d differs\n", k, p);
                ++bad;
            }
        }
    }
    printf("%s: n=%lld nnz=%lld d=%d K=%d, %d loopback ranks (hub rows %lld on rank 0, ghosts %lld), "
           "every hop %s the one-GPU hop\n", bad ? "FAIL" : "ok", (long long)n, (long long)nnz, d, K, P,
           (long long)info[0].hub_rows, (long long)info[0].n_ghost, bad ? "differs from" : "bitwise equal to");
    for (int p = 0; p < P; ++p) {
        srg_halo_share_destroy(share[p]);
        srg_halo_plan_destroy(plan[p]);
    }
    srg_comm_destroy(comm);
    return bad ? 1 : 0;
}
