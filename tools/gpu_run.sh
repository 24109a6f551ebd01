#!/bin/bash
# The one parametrised GPU launcher (every step under its own timeout; the first failure ends the call).
#
#   tools/gpu_run.sh tests OUT [pytest args...]    the given -m gpu tests (default: the whole suite), verbose log
#   tools/gpu_run.sh evidence OUT                  whole -m gpu suite + smoke + default bench (gpu_suite.sh), then the
#                                                  bench's kernel trace (profile.sh), then the 2-rank gloo rehearsal
#   tools/gpu_run.sh pmc OUT                       the PMC passes of the bench workload (profile.sh pmc)
#   tools/gpu_run.sh trace OUT LIB... [-- ARGS]    a kernel trace of the raster bench per library build, in the order
#                                                  given (DOGS_HIP_LIB; pass the list twice, reversed, for order effects);
#                                                  ARGS replace the bench's workload flags (e.g. --gaussians 5000000)
#   tools/gpu_run.sh ab OUT ROUNDS LIB...          interleaved bench A/B of library builds (abn.sh)
#   tools/gpu_run.sh bench OUT NAME [ARGS...]      one bench line (bench.py ARGS) into OUT/NAME.json
#   tools/gpu_run.sh train OUT [ARGS...]           tools/train_30k.py ARGS (config 2's schedule)
#
# Library variants for trace / ab are built beforehand on the CPU (tools/build_variant.sh).
set -e
CMD=$1; OUT=$2; shift 2
mkdir -p "$OUT"
export TMPDIR=/tmp
RASTER="--no-cpu-baseline --no-train-step --no-admm --no-sweep --no-reference-k"
case "$CMD" in
  tests)
    [ $# -gt 0 ] || set -- tests -m gpu
    timeout -k 10 ${TESTS_TIMEOUT:-900} python -u -m pytest "$@" -v -rA --timeout 400 --timeout-method thread \
        > "$OUT/tests.log" 2>&1 ;;
  evidence)
    bash tools/gpu_suite.sh "$OUT"
    bash tools/profile.sh "$OUT/prof"
    cp "$OUT"/prof/trace/*kernel_stats.csv "$OUT/" 2>/dev/null || true
    rm -rf "$OUT"/prof/trace/*kernel_trace.csv
    DOGS_DIST_BACKEND=gloo DOGS_BENCH_SHARE_DEVICE=1 timeout -k 10 400 python bench.py --gpus 2 --steps 10 --warmup 4 \
        --no-cpu-baseline --no-train-step > "$OUT/bench2.json" 2> "$OUT/bench2.err" ;;
  pmc)
    bash tools/profile.sh "$OUT/prof" pmc ;;
  trace)
    LIBS=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do LIBS+=("$1"); shift; done
    [ "$1" = "--" ] && shift
    ARGS=${*:-"--steps 20 --warmup 4"}
    for lib in "${LIBS[@]}"; do
      v=$(basename "$lib" .so); d="$OUT/$v"; i=1; while [ -e "$d" ]; do i=$((i + 1)); d="$OUT/$v.$i"; done
      DOGS_HIP_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$d" -o run -- \
          python3 bench.py $RASTER $ARGS > "$d.log" 2>&1
      rm -f "$d"/*kernel_trace.csv
    done ;;
  ab)
    bash tools/abn.sh "$OUT" "$@" ;;
  bench)
    NAME=$1; shift
    timeout -k 10 ${BENCH_TIMEOUT:-400} python bench.py "$@" > "$OUT/$NAME.json" 2> "$OUT/$NAME.err" ;;
  train)
    timeout -k 10 ${TRAIN_TIMEOUT:-900} python -u tools/train_30k.py --out "$OUT/run.json" "$@" > "$OUT/run.log" 2>&1 ;;
  *)
    echo "unknown command $CMD" >&2; exit 2 ;;
esac
