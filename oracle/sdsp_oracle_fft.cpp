// placeholder; filled in with the FFT restatement
