"""Generate the committed golden fixtures (run from the repo root).

* butter8_0p2_sos.json — cfg3's 4-section cascade, scipy.signal.butter(8, 0.2,
  output='sos'), rows [b0 b1 b2 a0 a1 a2].
The restatement-generated vectors (PFB / interpolator / FFT / channeliser,
which the reference's own tests do not pin) are produced by
make_vectors() from oracle/ and stored as .npz.
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def make_butter():
    from scipy import signal
    sos = signal.butter(8, 0.2, output="sos")
    with open(os.path.join(HERE, "butter8_0p2_sos.json"), "w") as f:
        json.dump({"source": "scipy.signal.butter(8, 0.2, output='sos')", "sos": sos.tolist()}, f, indent=1)


if __name__ == "__main__":
    make_butter()
