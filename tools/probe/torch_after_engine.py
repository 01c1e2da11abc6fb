"""Probe: does torch's HIP runtime come up after the engine's (two libamdhip64 in one process)?"""
import sys
sys.path.insert(0, ".")
import numpy as np
import veneur_amd as V

big = len(sys.argv) > 1 and sys.argv[1] == "big"
caps = (1, 1, 64, 100_000) if big else (1, 1, 64, 16)
rec = 10_000_000 if big else 1 << 17
with V.Engine(caps, max_batch_records=rec, max_batch_member_bytes=rec * 16) as e:
    e.ingest(set_hashes=(np.zeros(10, np.uint32), np.arange(10, dtype=np.uint64)))
    f = e.flush()
print("engine ok", f.set_estimate.tolist(), flush=True)
import torch
print("torch sees", torch.cuda.device_count(), flush=True)
print("available", torch.cuda.is_available(), flush=True)
x = torch.ones(4, device="cuda:0")
print("torch ok", x.sum().item(), flush=True)
