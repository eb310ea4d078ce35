set -u
mkdir -p gpurun_out/r3g
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3g/tests.log 2>&1 || { tail -30 gpurun_out/r3g/tests.log; exit 1; }
tail -1 gpurun_out/r3g/tests.log
PROF_TAG=r3g/hl bash tools/prof_headline.sh || exit 1
BENCH_EXTRA="--precision bf16 --no-f32-exact" PROF_TAG=r3g/bf16 bash tools/prof_headline.sh || exit 1
echo ok
