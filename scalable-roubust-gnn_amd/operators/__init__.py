"""Reference-compatible `operators` package (same module paths as SSRG/operators) backed by the
MI355X kernels of libsrgnn_hip.so.  Put `scalable-roubust-gnn_amd/` on sys.path in place of the
reference's `Scalable Spectral Robust GNN/` and models/ import it unchanged."""
