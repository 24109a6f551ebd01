set -o pipefail
mkdir -p gpurun_out/r2a
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2a/gpu_tests.log 2>&1 && \
timeout -k 10 400 python bench.py > gpurun_out/r2a/bench.json 2> gpurun_out/r2a/bench.err && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2a/smoke.log 2>&1 && \
bash tools/profile.sh gpurun_out/r2a/prof
