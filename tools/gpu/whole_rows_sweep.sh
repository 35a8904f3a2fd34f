O=gpurun_out/wr; mkdir -p $O
run() { env "$@" timeout -k 10 200 python tools/whole_rows_probe.py $WARGS >> $O/wr.jsonl 2>> $O/wr.err || exit 1; }
WARGS="" run SRGNN_X=0
WARGS="--u2 1" run SRGNN_X=0
WARGS="" run SRGNN_PACKED_U=8
WARGS="" run SRGNN_PACKED_ROWS=8
WARGS="" run SRGNN_PACKED_ROWS=2
WARGS="--natural" run SRGNN_X=0
