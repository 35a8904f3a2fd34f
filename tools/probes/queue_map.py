#!/usr/bin/env python3
"""Probe (run under rocprofv3 --kernel-trace): which hardware queue each kind of stream lands on.
A tiny fill kernel is launched on the default stream, on torch pool streams of normal and high
priority, and (through a hub-row SpMM) on the library's hub side stream; the trace's Queue_Id per
kernel shows which of them share a queue (sharing a queue serialises their kernels)."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "scalable-roubust-gnn_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from srgnn.csr import DeviceCSR  # noqa: E402
from srgnn.spmm import spmm  # noqa: E402

dev = torch.device("cuda", 0)
x = torch.zeros(1 << 20, device=dev)
marks = []


def tag(name, stream):
    with torch.cuda.stream(stream):
        for _ in range(int(name.split("#")[-1]) + 1 if "#" in name else 1):
            x.fill_(1.0)           # k instances: identify the stream by its kernel count
    marks.append(name)


x.fill_(0.0)                                    # default stream
torch.cuda.synchronize()
normal = [torch.cuda.Stream(dev) for _ in range(6)]
high = [torch.cuda.Stream(dev, priority=-1) for _ in range(6)]
print("default stream", torch.cuda.current_stream(dev).cuda_stream, flush=True)
for i, s in enumerate(normal):
    print(f"normal#{i}", s.cuda_stream, s.priority, flush=True)
for i, s in enumerate(high):
    print(f"high#{i}", s.cuda_stream, s.priority, flush=True)
# one hub row: the library forks its side stream
ip = np.array([0, 4096], dtype=np.int64)
A = DeviceCSR.from_tensors(ip, np.arange(4096, dtype=np.int32) % 64, np.ones(4096, np.float32), n_cols=64,
                           heavy_threshold=0, hub_threshold=0, device=dev)
spmm(A, torch.ones((64, 32), device=dev))
torch.cuda.synchronize()
for s in normal + high:
    with torch.cuda.stream(s):
        torch.cuda._sleep(1000)
torch.cuda.synchronize()
print("done", flush=True)
