"""STREAM-copy calibration of achievable HBM bandwidth (16 B per lane copy
kernel in libsdsp.so).  Prints GB/s counting read + write bytes."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import solid_dsp_amd as sd
    nbytes = 8 << 30
    a = torch.empty(nbytes // 4, dtype=torch.float32, device="cuda")
    b = torch.empty_like(a)
    a.fill_(1.0)
    s = torch.cuda.current_stream()
    L = sd.lib()
    for _ in range(3):
        L.sdsp_bandwidth_copy_device(a.data_ptr(), b.data_ptr(), nbytes, s.cuda_stream)
    ts = []
    for _ in range(10):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        L.sdsp_bandwidth_copy_device(a.data_ptr(), b.data_ptr(), nbytes, s.cuda_stream)
        e1.record(s)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ms = sorted(ts)[len(ts) // 2]
    print(json.dumps({"copy_bytes": nbytes, "median_ms": ms, "GBps_read_plus_write": 2 * nbytes / ms / 1e6}))


if __name__ == "__main__":
    main()
