"""Throughput of the reference-order (EXACT, default) c32 FIR and decimator kernels on
2^28 device-resident samples (cfg2 / cfg4 shapes): what an unchanged caller gets. Tools only."""
import sys, os, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
import solid_dsp_amd as sd
from solid_dsp_amd import DecimatingFIRFilter, FIRFilter
from solid_dsp_amd.filter import firdes
n = 1 << 28
res = {}
for name, mk in [("decim_exact_M32_L256_c32", lambda: DecimatingFIRFilter(firdes.firdes_kaiser(256, 1/64, 80.0, 0.0).astype(np.float32), np.float32(1/32), 32, sample_dtype=np.complex64, algo=sd.ALGO_EXACT)),
                 ("fir_exact_L256_c32", lambda: FIRFilter(firdes.firdes_kaiser(256, 0.1, 80.0, 0.0).astype(np.float32), np.float32(0.2), sample_dtype=np.complex64, algo=sd.ALGO_EXACT))]:
    f = mk()
    x = torch.randn(n, dtype=torch.complex64, device="cuda"); y = torch.empty(n, dtype=torch.complex64, device="cuda")
    st = torch.cuda.current_stream()
    for _ in range(2): f.execute_block_device(x, n, y, st)
    ts = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st); f.execute_block_device(x, n, y, st); e1.record(st); torch.cuda.synchronize(); ts.append(e0.elapsed_time(e1))
    ms = float(np.median(ts)); res[name] = {"ms_2^28": round(ms, 3), "GS/s": round(n / ms / 1e6, 1)}
print(json.dumps(res))
