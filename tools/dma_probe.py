"""Ingest rate into LDS on every CU: LDS-DMA vs register staging, L2-resident vs HBM source
(tools/dma_probe.hip).   python tools/dma_probe.py   -> one line per case, GB/s and B/clk/CU"""
import ctypes
import os
import subprocess
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "exp", "libdma_probe.so")
lib = ctypes.CDLL(LIB)
lib.dma_probe.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_ulonglong, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                          ctypes.c_void_p]
CUS = torch.cuda.get_device_properties(0).multi_processor_count
CLK = 2.1e9  # nominal shader clock for the per-CU figure (loaded parts run ~1.9-2.3 GHz)
sink = torch.zeros(4096, dtype=torch.int32, device="cuda")
s = torch.cuda.current_stream().cuda_stream
for region, label in ((1 << 20, "L2-resident 1 MiB"), (1 << 31, "HBM 2 GiB")):
    src = torch.randint(0, 255, (region,), dtype=torch.uint8, device="cuda")
    for blocks in (CUS * 2,):
        iters = 400 if region < (1 << 30) else 120
        for dma in (1, 0):
            for _ in range(2):
                lib.dma_probe(dma, src.data_ptr(), region - 1, iters, blocks, sink.data_ptr(), s)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                lib.dma_probe(dma, src.data_ptr(), region - 1, iters, blocks, sink.data_ptr(), s)
            e1.record()
            torch.cuda.synchronize()
            t = e0.elapsed_time(e1) / 5 * 1e-3
            byts = blocks * iters * 32768
            print(f"{label:18s} {'LDS-DMA' if dma else 'reg+ds_write':13s} blocks {blocks}: {byts / t / 1e9:8.1f} GB/s, "
                  f"{byts / t / CUS / CLK:6.1f} B/clk/CU", flush=True)
    del src
