/*
 * examples/cheby64_plan.c -- a plain C host of the fp64 Chebyshev steps (no Python, no torch): reads a CSR
 * file (the SRGCSR1 format of plan_propagate.c; its values, widened to fp64, are the operator's), then
 *   1. plans the operator for the fp64 steps: srg_plan_build over indptr / indices with NO fp32 values
 *      (SRG_PLAN_SPANS), for twice the panel width, block 0 split, whole hub rows above
 *      max(2048, nnz / 4096) entries (SRG_PLAN_WHOLE_HUBS) -- one plan serves every order and both L and F;
 *   2. runs an order-3 filter of two scales both ways -- srg_plan_cheby_step_f64 (column-blocked, hub
 *      workgroups beside) with the lean epilogue sequence, and srg_cheby_step_f64 (one launch per order,
 *      no schedule) with INIT + STEP -- and compares the two scales' outputs bit for bit;
 *   3. times one STEP order each way (HIP events over `reps` orders).
 * Prints one JSON line; exit status 0 = bitwise equal.  The reference's counterpart is pygsp's cheby_op
 * (SSRG/models/base_scalable/base_model.py:236-265), fp64.
 *
 *   examples/cheby64_plan <graph.csr> [d=64] [col_blocks=0 (automatic)] [reps=5]
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

static int read_all(FILE* f, void* p, size_t bytes)
{
    return fread(p, 1, bytes, f) == bytes ? 0 : 1;
}

/* the order-3 filter of two scales: R_s = (c0_s/2) T0 + c1_s T1 + c2_s T2 + c3_s T3, every order through
 * `plan` (lean sequence) or through srg_cheby_step_f64 (INIT, STEP, STEP); T: three work panels */
static int filter(srg_plan* plan, const int64_t* ip, const int32_t* ix, const double* v, int64_t n, int d,
                  const double* S, double* T[3], double* R, const double c[2][4], hipStream_t s)
{
    const double a1 = 1.0, a2 = 1.0;     /* the recurrence's shift and scale (any pair: both ways agree) */
    const int64_t rs = n * d;
    double c01[4] = {c[0][0], c[1][0], c[0][1], c[1][1]};   /* c0 then c1 per scale (STEP_FIRST) */
    double c0[2] = {c[0][0], c[1][0]}, c1[2] = {c[0][1], c[1][1]}, c2[2] = {c[0][2], c[1][2]},
           c3[2] = {c[0][3], c[1][3]};
    if (plan) {
        CHECK(srg_plan_cheby_step_f64(plan, v, S, NULL, T[0], d, d, SRG_CHEBY_INIT_T, a1, a2, NULL, NULL, 2, R, rs, s));
        CHECK(srg_plan_cheby_step_f64(plan, v, T[0], S, T[1], d, d, SRG_CHEBY_STEP_FIRST, a1, a2, c01, c2, 2, R, rs, s));
        CHECK(srg_plan_cheby_step_f64(plan, v, T[1], T[0], T[2], d, d, SRG_CHEBY_STEP | SRG_CHEBY_NO_T, a1, a2, NULL, c3,
                                      2, R, rs, s));
    } else {
        CHECK(srg_cheby_step_f64(ip, ix, v, n, NULL, S, NULL, T[0], d, d, SRG_CHEBY_INIT, a1, a2, c0, c1, 2, R, rs, s));
        CHECK(srg_cheby_step_f64(ip, ix, v, n, NULL, T[0], S, T[1], d, d, SRG_CHEBY_STEP, a1, a2, NULL, c2, 2, R, rs, s));
        CHECK(srg_cheby_step_f64(ip, ix, v, n, NULL, T[1], T[0], T[2], d, d, SRG_CHEBY_STEP, a1, a2, NULL, c3, 2, R, rs, s));
    }
    return 0;
}

int main(int argc, char** argv)
{
    if (argc < 2) {
        fprintf(stderr, "usage: %s <graph.csr> [d=64] [col_blocks=0] [reps=5]\n", argv[0]);
        return 1;
    }
    const int d = argc > 2 ? atoi(argv[2]) : 64;
    const int blocks = argc > 3 ? atoi(argv[3]) : 0;
    const int reps = argc > 4 ? atoi(argv[4]) : 5;
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
    float* vf = malloc(sizeof(float) * nnz);
    double* vd = malloc(sizeof(double) * nnz);
    if (!ip || !ix || !vf || !vd || read_all(f, ip, sizeof(int64_t) * (n + 1)) ||
        read_all(f, ix, sizeof(int32_t) * nnz) || read_all(f, vf, sizeof(float) * nnz)) {
        fprintf(stderr, "%s: short file\n", argv[1]);
        return 1;
    }
    fclose(f);
    for (int64_t j = 0; j < nnz; ++j) vd[j] = (double)vf[j];

    hipStream_t s;
    HCHECK(hipStreamCreate(&s));
    int64_t* d_ip;
    int32_t* d_ix;
    double *d_v, *buf;
    HCHECK(hipMalloc((void**)&d_ip, sizeof(int64_t) * (n + 1)));
    HCHECK(hipMalloc((void**)&d_ix, sizeof(int32_t) * nnz));
    HCHECK(hipMalloc((void**)&d_v, sizeof(double) * nnz));
    HCHECK(hipMemcpy(d_ip, ip, sizeof(int64_t) * (n + 1), hipMemcpyHostToDevice));
    HCHECK(hipMemcpy(d_ix, ix, sizeof(int32_t) * nnz, hipMemcpyHostToDevice));
    HCHECK(hipMemcpy(d_v, vd, sizeof(double) * nnz, hipMemcpyHostToDevice));
    CHECK(srg_csr_validate(d_ip, d_ix, n, nnz, n, s));

    /* S, three work panels and two scales' outputs, each way */
    const size_t panel = (size_t)n * d;
    HCHECK(hipMalloc((void**)&buf, sizeof(double) * panel * 11));
    double* S = buf;
    double* Tp[3] = {buf + panel, buf + 2 * panel, buf + 3 * panel};
    double* To1[3] = {buf + 4 * panel, buf + 5 * panel, buf + 6 * panel};
    double* Rp = buf + 7 * panel;
    double* R1 = buf + 9 * panel;
    double* hs = malloc(sizeof(double) * panel);
    uint64_t r = 0x9e3779b97f4a7c15ull;
    for (size_t i = 0; i < panel; ++i) {
        r ^= r << 13; r ^= r >> 7; r ^= r << 17;
        hs[i] = (double)(r >> 11) / 9007199254740992.0 * 2.0 - 1.0;
    }
    HCHECK(hipMemcpy(S, hs, sizeof(double) * panel, hipMemcpyHostToDevice));
    const double c[2][4] = {{1.3, -0.7, 0.25, -0.05}, {0.9, 0.4, 0.1, 0.02}};

    /* 1. the plan */
    const int64_t hub_t = nnz / 4096 > 2048 ? nnz / 4096 : 2048;
    HCHECK(hipStreamSynchronize(s));
    const double t0 = now_ms();
    srg_plan* P = NULL;
    CHECK(srg_plan_build(d_ip, d_ix, NULL, n, 2 * d, 1 << 20, blocks, hub_t, SRG_PLAN_NONE,
                         SRG_PLAN_SPANS | SRG_PLAN_SPLIT_BLOCK0 | SRG_PLAN_WHOLE_HUBS, s, &P));
    HCHECK(hipStreamSynchronize(s));
    const double build_ms = now_ms() - t0;
    srg_plan_desc desc;
    CHECK(srg_plan_describe(P, &desc));

    /* 2. both ways, bit for bit */
    if (filter(P, d_ip, d_ix, d_v, n, d, S, Tp, Rp, c, s)) return 2;
    if (filter(NULL, d_ip, d_ix, d_v, n, d, S, To1, R1, c, s)) return 2;
    HCHECK(hipStreamSynchronize(s));
    double* hp = malloc(sizeof(double) * panel * 2);
    double* h1 = malloc(sizeof(double) * panel * 2);
    HCHECK(hipMemcpy(hp, Rp, sizeof(double) * panel * 2, hipMemcpyDeviceToHost));
    HCHECK(hipMemcpy(h1, R1, sizeof(double) * panel * 2, hipMemcpyDeviceToHost));
    const int same = memcmp(hp, h1, sizeof(double) * panel * 2) == 0;

    /* 3. one STEP order each way */
    hipEvent_t e0, e1;
    HCHECK(hipEventCreate(&e0));
    HCHECK(hipEventCreate(&e1));
    const double c2[2] = {c[0][2], c[1][2]};
    float ms_plan = 0.f, ms_one = 0.f;
    HCHECK(hipEventRecord(e0, s));
    for (int i = 0; i < reps; ++i)
        CHECK(srg_plan_cheby_step_f64(P, d_v, Tp[0], S, Tp[1], d, d, SRG_CHEBY_STEP, 1.0, 1.0, NULL, c2, 2, Rp,
                                      (int64_t)panel, s));
    HCHECK(hipEventRecord(e1, s));
    HCHECK(hipEventSynchronize(e1));
    HCHECK(hipEventElapsedTime(&ms_plan, e0, e1));
    HCHECK(hipEventRecord(e0, s));
    for (int i = 0; i < reps; ++i)
        CHECK(srg_cheby_step_f64(d_ip, d_ix, d_v, n, NULL, To1[0], S, To1[1], d, d, SRG_CHEBY_STEP, 1.0, 1.0, NULL, c2,
                                 2, R1, (int64_t)panel, s));
    HCHECK(hipEventRecord(e1, s));
    HCHECK(hipEventSynchronize(e1));
    HCHECK(hipEventElapsedTime(&ms_one, e0, e1));
    CHECK(srg_plan_destroy(P, s));

    printf("{\"n\": %lld, \"nnz\": %lld, \"d\": %d, \"col_blocks\": %d, \"n_launch\": %d, \"hub_rows_whole\": %d, "
           "\"plan_bytes\": %lld, \"build_ms\": %.3f, \"ms_per_step_plan\": %.4f, \"ms_per_step_one_launch\": %.4f, "
           "\"bitwise_vs_one_launch\": %s}\n",
           (long long)n, (long long)nnz, d, desc.col_blocks, desc.n_launch, desc.hub_rows_whole,
           (long long)desc.device_bytes, build_ms, ms_plan / reps, ms_one / reps, same ? "true" : "false");
    free(ip); free(ix); free(vf); free(vd); free(hs); free(hp); free(h1);
    HCHECK(hipFree(buf));
    HCHECK(hipFree(d_ip));
    HCHECK(hipFree(d_ix));
    HCHECK(hipFree(d_v));
    return same ? 0 : 3;
}
