#!/bin/bash
# Parameterised same-box A/B of compile-time variants of the product library (replaces the
# per-session scripts of rounds 2-3).  Variants are built beforehand on the CPU host:
#   scripts/build_variant.sh NAME "-DMACRO=VALUE ..."  ->  chunker_amd/_ab/libchunker_amd_NAME.so
# then, on the GPU box:
#   VARIANTS="prod NAME" CONFIGS="c2 c4" ROUNDS=3 TAG=r04_x bash scripts/gpu_ab.sh
# Environment:
#   VARIANTS   product = "prod", others = library names under chunker_amd/_ab (required);
#              "+FLAG[,FLAG...]" = the product library with those bench.py flags
#              (e.g. "+--no-overlap", "+--split-mode=1,--bound-cus=32")
#   CONFIGS    bench.py configs to alternate (default "c2")
#   ROUNDS     alternating rounds (default 3)
#   STEPS      bench.py --steps (default 8)
#   TESTS      pytest node ids run on every non-prod variant first (default: the parity,
#              config and fuzz GPU suites); TESTS=none skips them
#   TAG        output prefix under gpurun_out/ (default ab)
# Output: gpurun_out/${TAG}_ab.txt, one line per run: config variant round value digest_ms scan_ms.
# Every GPU step has its own time limit and the first failure ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
: "${VARIANTS:?set VARIANTS}"
CONFIGS=${CONFIGS:-c2}
ROUNDS=${ROUNDS:-3}
STEPS=${STEPS:-8}
TAG=${TAG:-ab}
TESTS=${TESTS:-"tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_fuzz.py"}
lib_of() { case "$1" in prod|+*) echo "" ;; *) echo "chunker_amd/_ab/libchunker_amd_$1.so" ;; esac; }
flag_of() { case "$1" in +*) echo "${1#+}" | tr ',' ' ' ;; *) echo "" ;; esac; }
if [ "$TESTS" != none ]; then
  for v in $VARIANTS; do
    case "$v" in prod|+*) continue ;; esac
    CHUNKER_AMD_LIB=$(lib_of "$v") timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread \
      -m gpu $TESTS > "gpurun_out/${TAG}_${v}_tests.log" 2>&1 || { tail -30 "gpurun_out/${TAG}_${v}_tests.log"; exit 1; }
    echo "$v tests: $(tail -1 "gpurun_out/${TAG}_${v}_tests.log")"
  done
fi
for r in $(seq 1 "$ROUNDS"); do
  for cfg in $CONFIGS; do
    for v in $VARIANTS; do
      out="gpurun_out/${TAG}_${cfg}_$(echo "$v" | tr -c 'A-Za-z0-9_\n' _)_$r.json"
      CHUNKER_AMD_LIB=$(lib_of "$v") timeout -k 10 300 python3 bench.py --config "$cfg" --steps "$STEPS" --warmup 2 \
        --no-cpu-baseline --no-concurrent --no-clock --e2e '' --drop-in '' $(flag_of "$v") > "$out" 2> "${out%.json}.err" || { tail -3 "${out%.json}.err"; exit 1; }
      python3 -c "
import json; l = json.loads(open('$out').read().strip().splitlines()[-1])
print('$cfg', '$v', $r, l['value'], l['ms_per_step'], l['stages_ms']['digest_timed'], l['stages_ms']['scan'])" | tee -a "gpurun_out/${TAG}_ab.txt"
    done
  done
done
echo "rc=0"
