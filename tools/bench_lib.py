"""bench.py against another build of libsdsp.so (alternating A/B runs of whole bench lines on
one box):  python tools/bench_lib.py LIB.so --config 6 --steps 20 --warmup 5 --no-cpu"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    lib = os.path.abspath(sys.argv[1])
    import solid_dsp_amd._lib as LL
    LL.LIB_PATH = lib
    sys.argv = [os.path.join(REPO, "bench.py")] + sys.argv[2:]
    import bench
    bench.main()


if __name__ == "__main__":
    main()
