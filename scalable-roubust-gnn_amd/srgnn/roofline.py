"""Byte models of SURVEY.md §8(d) for one hop Y = Â X (fp32 features, int32 ids, fp32 values).

no-reuse ("algorithmic") bytes, the figure roofline.achieved is computed from:
    B_hop = nnz * (4 value + 4 column id + 4 d gathered X row) + (N + 1) * s_ptr + N * 4 d (Y write)
compulsory bytes (every byte touched once):
    nnz * 8 + (N + 1) * s_ptr + 2 * N * 4 d
s_ptr = 4 when nnz < 2^31 (the reference's int32 indptr), else 8.  Our kernels read int64 row
pointers; the model keeps the survey's definition so numbers compare across implementations.
"""
MI355X_HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md chip table (8.0 TB/s spec)
MI355X_HBM_MEASURED_GBS = 6290.0      # ditto, float4 copy
# 2 * FETCH_SIZE over the bytes a random-row gather asks for (tools/spmm_probe.py --permutation at the
# products size, d = 128: profiles/r04_pmc_gather_calibration.txt); reads / this = calibrated reads
PMC_READ_CALIBRATION = 1.038


def s_ptr(nnz: int) -> int:
    return 4 if nnz < 2 ** 31 else 8


def bytes_no_reuse(n_rows: int, nnz: int, d: int) -> int:
    return nnz * (4 + 4 + 4 * d) + (n_rows + 1) * s_ptr(nnz) + n_rows * 4 * d


def bytes_compulsory(n_rows: int, nnz: int, d: int, n_cols: int | None = None) -> int:
    n_cols = n_rows if n_cols is None else n_cols
    return nnz * 8 + (n_rows + 1) * s_ptr(nnz) + n_rows * 4 * d + n_cols * 4 * d


def cheby_step_bytes_no_reuse_f64(n_rows: int, nnz: int, d: int, n_scales: int) -> int:
    """One fp64 Chebyshev STEP launch (srg_cheby_step_f64: T_{k+1} = F T_k - T_{k-1}, R_s += c_s T_{k+1}),
    pygsp cheby_op's precision: the SpMM with fp64 values and gathered rows (8 B) plus the epilogue's
    panel passes -- T_{k-1} read, T_{k+1} written, every scale's R read and written."""
    return nnz * (4 + 8 + 8 * d) + (n_rows + 1) * 8 + n_rows * 8 * d * (2 + 2 * n_scales)


def cheby_step_bytes_compulsory_f64(n_rows: int, nnz: int, d: int, n_scales: int) -> int:
    """cheby_step_bytes_no_reuse_f64 with T_k read once."""
    return nnz * (4 + 8) + (n_rows + 1) * 8 + n_rows * 8 * d * (3 + 2 * n_scales)
