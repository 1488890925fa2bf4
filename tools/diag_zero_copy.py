"""Diagnostic: does torch.as_tensor(__cuda_array_interface__) view libcbgpu results without a copy, and
does the view keep the result alive?  usage: python tools/diag_zero_copy.py"""
import gc
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "tests"))
import combblas_amd as cb  # noqa: E402
from combblas_amd import dist as cbd  # noqa: E402
from dist_support import random_csc  # noqa: E402

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29677")
dist.init_process_group("gloo", rank=0, world_size=1)
ctx = cb.Context(0)
be = cbd.GpuBackend(ctx)
A = random_csc(300, 280, 0.03, 1)
B = random_csc(280, 260, 0.03, 2)
bA = cbd.block_from_host(300, 280, A.indptr, A.indices, A.data, be.device)
bB = cbd.block_from_host(280, 260, B.indptr, B.indices, B.data, be.device)
R = (A @ B).tocsc()
R.sort_indices()
C1 = be.multiply(bA, bB, cb.PlusTimesSRing("f64"))
print("zero-copy owner attached:", hasattr(C1.cp, "__cuda_array_interface__"), "cp ptr", hex(C1.cp.data_ptr()))
ok1 = np.array_equal(C1.cp.cpu().numpy(), R.indptr) and np.array_equal(C1.ir.cpu().numpy(), R.indices)
gc.collect()
outs = [be.multiply(bB.__class__(280, 260, bB.cp, bB.ir, bB.val), bB, cb.PlusTimesSRing("f64"))
        if False else be.multiply(bA, bB, cb.PlusTimesSRing("f64")) for _ in range(5)]
gc.collect()
torch.cuda.synchronize()
ok2 = np.array_equal(C1.cp.cpu().numpy(), R.indptr) and np.array_equal(C1.ir.cpu().numpy(), R.indices) \
    and np.array_equal(C1.val.cpu().numpy(), R.data)
print("first result correct:", ok1, "still correct after 5 more products:", ok2)
print("ptrs:", [hex(o.cp.data_ptr()) for o in outs])
dist.destroy_process_group()
