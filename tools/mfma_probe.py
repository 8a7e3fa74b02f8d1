"""Run tools/mfma_probe.hip: fp32 MFMA TFLOP/s from registers and from the LDS slice loop."""
import ctypes
import os
import subprocess

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "mfma_probe.so")
if not os.path.exists(SO):
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "-shared", "--offload-arch=gfx950",
                    "-I" + os.path.join(HERE, "..", "include"), os.path.join(HERE, "mfma_probe.hip"), "-o", SO], check=True)
lib = ctypes.CDLL(SO)
lib.probe_run.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
g = torch.randn(8192 * 768 + 4096, device='cuda')
out = torch.zeros(1024, device="cuda")
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
flops_per_iter = {0: 4 * 4096, 1: 48 * 4096, 2: 48 * 4096, 3: 48 * 4096, 4: 48 * 4096}  # per wave
for which, name in [(0, "regs 4acc"), (1, "lds only"), (2, "+barrier"), (3, "+ds_write"), (4, "+global")]:
    for blocks in (512,):
        iters = 20000 if which == 0 else 1500
        lib.probe_run(which, blocks, 10, ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(g.data_ptr()), st)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        lib.probe_run(which, blocks, iters, ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(g.data_ptr()), st)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1)
        tf = blocks * 4 * iters * flops_per_iter[which] / ms / 1e9
        print("%-12s blocks %5d: %.1f TFLOP/s (%.3f ms)" % (name, blocks, tf, ms))
