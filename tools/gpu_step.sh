# one gpurun call: the GPU tests named in $TESTS (default: all), then bench.py with $BENCH_ARGS, each under its own limit
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu ${TESTS:-tests} > gpurun_out/tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/tests.log; exit 1; }
tail -3 gpurun_out/tests.log
if [ -n "${BENCH_ARGS+x}" ]; then
  timeout -k 10 900 python bench.py $BENCH_ARGS > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -30 gpurun_out/bench.err; exit 1; }
  tail -c 400 gpurun_out/bench.json
fi
