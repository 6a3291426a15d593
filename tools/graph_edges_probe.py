"""Probe: which dependencies does a HIP stream capture record when a side stream waits on the
capturing stream twice?  Dumps the captured graph (DOT) and prints the kernel-node edges.
    python tools/graph_edges_probe.py"""
import re

import torch

A = torch.cuda.Stream()
B = torch.cuda.Stream()
x = torch.zeros(4, device="cuda")
y = torch.zeros(4, device="cuda")
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
g.enable_debug_mode()
with torch.cuda.graph(g, stream=A):
    B.wait_stream(A)
    with torch.cuda.stream(B):
        x.add_(1.0)          # k1 (side)
    y.add_(2.0)              # kA (main)
    B.wait_stream(A)
    with torch.cuda.stream(B):
        x.mul_(3.0)          # k2 (side): must follow k1 and kA
    A.wait_stream(B)
    y.add_(x)                # kJ (main, after the join)
g.debug_dump("gpurun_out/probe_graph.dot")
txt = open("gpurun_out/probe_graph.dot").read()
print(txt[:4000])
g.replay()
torch.cuda.synchronize()
print("x", x.tolist(), "y", y.tolist())
