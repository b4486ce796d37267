# cfg8 pass-kernel lab (tools/fft_lab.py over tools/_build/libsdsp_lab.so) under a
# kernel trace, so each variant's column / row pass durations are separable:
#   gpurun -- 'bash tools/gpu_fftlab.sh TAG'   (FFT_CASES as in tools/fft_lab.py)
set -o pipefail
TAG=${1:-fftlab}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
FFT_CASES=${FFT_CASES:-16,128,256,384} FFT_BURST=${FFT_BURST:-10} FFT_ROUNDS=${FFT_ROUNDS:-15} \
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- \
  python -u tools/fft_lab.py > gpurun_out/${TAG}.log 2>&1
rc=$?; echo "== $TAG rc=$rc"; tail -40 gpurun_out/${TAG}.log; exit $rc
