/*
 * examples/plan_propagate.c -- a plain C host of the one-GPU planner (no Python, no torch): reads a CSR
 * file (tools/dump_graph.py writes the bench's workloads), then
 *   1. the reference's call pattern -- GraphOp.propagate(K) once per run (SSRG/tasks/
 *      node_classification.py:62): a fresh plan for K hops, the K hops, the plan released -- timed
 *      with the host clock (twice: the first run warms the code objects and the memory pool);
 *   2. a long-lived plan for many runs (compact launch-ordered copies): build time, then `reps` runs
 *      of K hops between HIP events -> ms per hop;
 *   3. hops 1, 2 and K compared bit for bit with the unscheduled one-launch hops (srg_spmm_csr_f32,
 *      no row order: a different kernel path over the caller's CSR).
 * Prints one JSON line; exit status 0 = bitwise equal.
 *
 *   examples/plan_propagate <graph.csr> [d=128] [K=10] [reps=10]
 */
#define _POSIX_C_SOURCE 199309L
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

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

static double now_ms(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec * 1e3 + t.tv_nsec * 1e-6;
}

static double g_t0;
static void stage(const char* what)
{
    fprintf(stderr, "[%9.1f ms] %s\n", now_ms() - g_t0, what);
    fflush(stderr);
}

static int read_all(FILE* f, void* p, size_t bytes)
{
    return fread(p, 1, bytes, f) == bytes ? 0 : 1;
}

/* The plan's launches checked on the host before any hop runs: schedules name rows in [0, n), every
 * span lies in [0, nnz] with beg <= end, and the row-indexed spans of the scheduled rows are the
 * slot spans.  Returns the number of violations. */
static long validate(srg_plan* P, int64_t n, int64_t nnz, int d)
{
    srg_plan_desc desc;
    if (srg_plan_describe(P, &desc)) return -1;
    long bad = 0;
    for (int i = 0; i < desc.n_launch; ++i) {
        srg_hop_launch L;
        int32_t join = 0;
        if (srg_plan_launch(P, i, d, &L, &join, NULL)) return -1;
        if (L.n_rows < 0 || L.n_rows > n || L.n_hub + L.n_heavy > L.n_rows) { ++bad; continue; }
        if (!L.n_rows) continue;
        int32_t* order = malloc(sizeof(int32_t) * L.n_rows);
        int64_t* sb = malloc(sizeof(int64_t) * L.n_rows);
        int64_t* se = malloc(sizeof(int64_t) * L.n_rows);
        int64_t* rb = malloc(sizeof(int64_t) * (n + 1));
        int64_t* re = malloc(sizeof(int64_t) * n);
        hipMemcpy(order, L.row_order, sizeof(int32_t) * L.n_rows, hipMemcpyDeviceToHost);
        hipMemcpy(rb, L.row_beg, sizeof(int64_t) * (L.row_end ? n : n + 1), hipMemcpyDeviceToHost);
        if (L.row_end) hipMemcpy(re, L.row_end, sizeof(int64_t) * n, hipMemcpyDeviceToHost);
        if (L.slot_beg) {
            hipMemcpy(sb, L.slot_beg, sizeof(int64_t) * L.n_rows, hipMemcpyDeviceToHost);
            hipMemcpy(se, L.slot_end, sizeof(int64_t) * L.n_rows, hipMemcpyDeviceToHost);
        }
        for (int64_t j = 0; j < L.n_rows; ++j) {
            const int32_t r = order[j];
            if (r < 0 || r >= n) { ++bad; continue; }
            const int64_t b = rb[r], e = L.row_end ? re[r] : rb[r + 1];
            if (b < 0 || e < b || e > nnz) ++bad;
            if (L.slot_beg && (sb[j] != b || se[j] != e)) ++bad;
        }
        if (bad) fprintf(stderr, "launch %d: %ld bad spans or rows\n", i, bad);
        free(order); free(sb); free(se); free(rb); free(re);
    }
    return bad;
}

int main(int argc, char** argv)
{
    if (argc < 2) {
        fprintf(stderr, "usage: %s <graph.csr> [d=128] [K=10] [reps=10]\n", argv[0]);
        return 1;
    }
    const int d = argc > 2 ? atoi(argv[2]) : 128;
    const int K = argc > 3 ? atoi(argv[3]) : 10;
    const int reps = argc > 4 ? atoi(argv[4]) : 10;
    g_t0 = now_ms();
    FILE* f = fopen(argv[1], "rb");
    if (!f) { perror(argv[1]); return 1; }
    char magic[8];
    int64_t hdr[2];
    if (read_all(f, magic, 8) || memcmp(magic, "SRGCSR1", 8) || read_all(f, hdr, sizeof(hdr))) {
        fprintf(stderr, "%s: not a SRGCSR1 file\n", argv[1]);
        return 1;
    }
    const int64_t n = hdr[0], nnz = hdr[1];
    int64_t* ip = malloc(sizeof(int64_t) * (n + 1));
    int32_t* ix = malloc(sizeof(int32_t) * nnz);
    float* vv = malloc(sizeof(float) * nnz);
    if (!ip || !ix || !vv || read_all(f, ip, sizeof(int64_t) * (n + 1)) || read_all(f, ix, sizeof(int32_t) * nnz) ||
        read_all(f, vv, sizeof(float) * nnz)) {
        fprintf(stderr, "%s: short file\n", argv[1]);
        return 1;
    }
    fclose(f);
    stage("read");

    hipStream_t s;
    HCHECK(hipStreamCreate(&s));
    int64_t *d_ip;
    int32_t *d_ix;
    float *d_v, *buf;
    HCHECK(hipMalloc((void**)&d_ip, sizeof(int64_t) * (n + 1)));
    HCHECK(hipMalloc((void**)&d_ix, sizeof(int32_t) * nnz));
    HCHECK(hipMalloc((void**)&d_v, sizeof(float) * nnz));
    HCHECK(hipMemcpy(d_ip, ip, sizeof(int64_t) * (n + 1), hipMemcpyHostToDevice));
    HCHECK(hipMemcpy(d_ix, ix, sizeof(int32_t) * nnz, hipMemcpyHostToDevice));
    HCHECK(hipMemcpy(d_v, vv, sizeof(float) * nnz, hipMemcpyHostToDevice));
    free(ix);
    free(vv);
    CHECK(srg_csr_validate(d_ip, d_ix, n, nnz, n, s));
    stage("uploaded, validated");

    /* K + 1 panels of n x d, X = U[-1, 1) */
    const size_t panel = (size_t)n * d;
    HCHECK(hipMalloc((void**)&buf, sizeof(float) * panel * (K + 1)));
    float** panels = malloc(sizeof(float*) * (K + 1));
    for (int k = 0; k <= K; ++k) panels[k] = buf + (size_t)k * panel;
    float* hx = malloc(sizeof(float) * panel);
    uint64_t r = 0x9e3779b97f4a7c15ull;
    for (size_t i = 0; i < panel; ++i) {
        r ^= r << 13; r ^= r >> 7; r ^= r << 17;
        hx[i] = (float)((double)(r >> 11) / 9007199254740992.0 * 2.0 - 1.0);
    }
    HCHECK(hipMemcpy(panels[0], hx, sizeof(float) * panel, hipMemcpyHostToDevice));
    stage("features");

    /* 0. two plans for K hops checked on the host and run, with a synchronisation after each step */
    for (int t = 0; t < 2; ++t) {
        srg_plan* P0 = NULL;
        CHECK(srg_plan_build(d_ip, d_ix, d_v, n, d, K, 0, SRG_PLAN_AUTO, SRG_PLAN_AUTO, 0, s, &P0));
        HCHECK(hipStreamSynchronize(s));
        const long bad = validate(P0, n, nnz, d);
        if (bad) { fprintf(stderr, "plan layout invalid (%ld)\n", bad); return 4; }
        stage("plan checked");
        CHECK(srg_plan_propagate_f32(P0, panels, d, d, 1, 0, s));
        HCHECK(hipStreamSynchronize(s));
        stage("one hop");
        CHECK(srg_plan_propagate_f32(P0, panels, d, d, K, 0, s));
        HCHECK(hipStreamSynchronize(s));
        stage("K hops");
        CHECK(srg_plan_destroy(P0, s));
        HCHECK(hipStreamSynchronize(s));
        stage("plan released");
    }

    /* 1. one propagate(K) as the reference runs it: plan + hops + release */
    double one_shot = 0.0;
    for (int t = 0; t < 2; ++t) {
        HCHECK(hipStreamSynchronize(s));
        const double t0 = now_ms();
        srg_plan* P1 = NULL;
        CHECK(srg_plan_build(d_ip, d_ix, d_v, n, d, K, 0, SRG_PLAN_AUTO, SRG_PLAN_AUTO, 0, s, &P1));
        stage("one-shot plan built");
        CHECK(srg_plan_propagate_f32(P1, panels, d, d, K, 0, s));
        CHECK(srg_plan_destroy(P1, s));
        HCHECK(hipStreamSynchronize(s));
        one_shot = now_ms() - t0;
        stage("one-shot hops done");
    }

    /* 2. a long-lived plan */
    HCHECK(hipStreamSynchronize(s));
    double t0 = now_ms();
    srg_plan* P = NULL;
    CHECK(srg_plan_build(d_ip, d_ix, d_v, n, d, K * (reps + 1), 0, SRG_PLAN_AUTO, SRG_PLAN_AUTO, 0, s, &P));
    HCHECK(hipStreamSynchronize(s));
    const double build_ms = now_ms() - t0;
    stage("long-lived plan built");
    srg_plan_desc desc;
    CHECK(srg_plan_describe(P, &desc));
    CHECK(srg_plan_propagate_f32(P, panels, d, d, K, 0, s));   /* warm */
    hipEvent_t e0, e1;
    HCHECK(hipEventCreate(&e0));
    HCHECK(hipEventCreate(&e1));
    HCHECK(hipEventRecord(e0, s));
    for (int i = 0; i < reps; ++i) CHECK(srg_plan_propagate_f32(P, panels, d, d, K, 0, s));
    HCHECK(hipEventRecord(e1, s));
    HCHECK(hipEventSynchronize(e1));
    float loop_ms = 0.0f;
    HCHECK(hipEventElapsedTime(&loop_ms, e0, e1));
    stage("timed hops done");

    /* 3. hops 1, 2, K against the unscheduled one-launch hops */
    float *ref, *ref2;
    HCHECK(hipMalloc((void**)&ref, sizeof(float) * panel));
    HCHECK(hipMalloc((void**)&ref2, sizeof(float) * panel));
    float* hy = malloc(sizeof(float) * panel);
    int bitwise = 1;
    const float* src = panels[0];
    for (int k = 1; k <= K; ++k) {
        float* dst = (k & 1) ? ref : ref2;
        CHECK(srg_spmm_csr_f32(d_ip, d_ix, d_v, n, NULL, 0, 0, src, d, dst, d, d, 0, s));
        src = dst;
        if (k == 1 || k == 2 || k == K) {
            HCHECK(hipMemcpyAsync(hx, dst, sizeof(float) * panel, hipMemcpyDeviceToHost, s));
            HCHECK(hipMemcpyAsync(hy, panels[k], sizeof(float) * panel, hipMemcpyDeviceToHost, s));
            HCHECK(hipStreamSynchronize(s));
            stage("compared a hop");
            if (memcmp(hx, hy, sizeof(float) * panel)) {
                bitwise = 0;
                fprintf(stderr, "hop %d differs from the one-launch hop\n", k);
            }
        }
    }
    printf("{\"example\": \"plan_propagate\", \"graph\": \"%s\", \"n\": %lld, \"nnz\": %lld, \"d\": %d, \"K\": %d, "
           "\"col_blocks\": %d, \"launches_per_hop\": %d, \"compact\": %d, \"split_block0\": %d, \"hub_chain\": %d, "
           "\"plan_device_bytes\": %lld, \"build_ms_long_lived\": %.3f, \"ms_per_hop\": %.4f, \"reps\": %d, "
           "\"one_shot_ms_total\": %.3f, \"one_shot_ms_per_hop\": %.4f, \"bitwise_vs_one_launch\": %s}\n",
           argv[1], (long long)n, (long long)nnz, d, K, desc.col_blocks, desc.n_launch, desc.compact,
           desc.split_block0, desc.hub_chain, (long long)desc.device_bytes, build_ms, loop_ms / (reps * K), reps,
           one_shot, one_shot / K, bitwise ? "true" : "false");
    CHECK(srg_plan_destroy(P, s));
    HCHECK(hipStreamSynchronize(s));
    hipFree(ref);
    hipFree(ref2);
    hipFree(buf);
    hipFree(d_ip);
    hipFree(d_ix);
    hipFree(d_v);
    free(hx);
    free(hy);
    free(ip);
    free(panels);
    return bitwise ? 0 : 3;
}
