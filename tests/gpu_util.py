"""Helpers for the -m gpu parity tests (device buffers through torch, which is
plumbing only: allocation, streams, events)."""
import numpy as np

_TORCH_DT = None


def torch_dtype(np_dt):
    import torch
    return {np.dtype(np.float32): torch.float32, np.dtype(np.float64): torch.float64,
            np.dtype(np.complex64): torch.complex64, np.dtype(np.complex128): torch.complex128}[np.dtype(np_dt)]


def to_dev(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).to("cuda")


def empty_dev(n, np_dt):
    import torch
    return torch.empty(n, dtype=torch_dtype(np_dt), device="cuda")


def to_host(t):
    import torch
    torch.cuda.synchronize()
    return t.cpu().numpy()


def rel_rms(y, ref):
    y = np.asarray(y, dtype=np.complex128)
    ref = np.asarray(ref, dtype=np.complex128)
    return float(np.linalg.norm(y - ref) / max(np.linalg.norm(ref), 1e-300))


def bits_equal(a, b):
    a = np.ascontiguousarray(a)
    b = np.ascontiguousarray(b)
    if a.shape != b.shape or a.dtype != b.dtype:
        return False
    return a.view(np.uint8).tobytes() == b.view(np.uint8).tobytes()
