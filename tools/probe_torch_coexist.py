"""Probe: can torch's bundled HIP runtime and libmtgpu.so (ROCm 7.2 runtime) share a process?"""
import torch
x = torch.ones(1024, device="cuda:0")
torch.cuda.synchronize()
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fluidframework_amd.engine import Engine
e = Engine(4, rows_per_doc=1024)
e.open_docs(0, 4)
e.sync()
print("engine status", e.status(range(4)))
y = x * 2
torch.cuda.synchronize()
print("torch after engine OK", float(y.sum()))
