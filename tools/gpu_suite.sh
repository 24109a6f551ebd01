#!/bin/bash
# One GPU call: the whole -m gpu suite (no -x: every result is recorded), smoke, then the default bench line.
# usage: tools/gpu_suite.sh OUTDIR [pytest args...]
OUT=${1:-gpurun_out/suite}; shift
mkdir -p "$OUT"
export TMPDIR=/tmp DOGS_TEST_LOG="$OUT/fullsize.jsonl"
( while true; do date +%T >> "$OUT/heartbeat"; sleep 50; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 ${SUITE_TIMEOUT:-700} python -u -m pytest tests -m gpu -v -rA --timeout 400 --timeout-method thread "$@" > "$OUT/gpu_tests.log" 2>&1
rc=$?
echo "pytest rc=$rc" >> "$OUT/gpu_tests.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi   # a crash / timeout: nothing more on the GPU
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit $?
timeout -k 10 ${BENCH_TIMEOUT:-300} python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
