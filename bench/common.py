"""Shared helpers for the BASELINE config benchmarks."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

FP32_PEAK_TFLOPS = 157.3      # MI355X vector/matrix fp32 (spec)
BF16_PEAK_TFLOPS = 2500.0     # dense (spec)
HBM_TBPS = 6.3                # achievable
PCIE_GBPS = 63.0              # Gen5 x16 spec


def sync():
    try:
        import torch
        if torch.cuda.is_available():
            torch.cuda.synchronize()
    except Exception:
        pass


def timeit(fn, reps: int, warmup: int = 2) -> float:
    """Mean milliseconds per call."""
    for _ in range(warmup):
        fn()
    sync()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    sync()
    return (time.perf_counter() - t) * 1e3 / reps


def emit(obj) -> None:
    print(json.dumps(obj), flush=True)
