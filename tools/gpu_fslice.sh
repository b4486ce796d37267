# cfg8 batch slices under a kernel trace (tools/fft_slice_ab.py): per-transform column / row pass
# times when each slice's intermediate was written just before (Infinity-Cache question,
# profiles/r06/LAB.md):  gpurun -- 'bash tools/gpu_fslice.sh'
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
FFT_SLICES=0,8,16 FFT_ROUNDS=5 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fslice -o run -- python tools/fft_slice_ab.py > gpurun_out/fslice.log 2>&1
