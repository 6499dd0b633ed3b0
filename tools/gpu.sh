#!/bin/bash
# GPU-box recipes (one gpurun call runs any sequence of them):
#   bash tools/gpu.sh TAG STEP [STEP ...]
# Each GPU step has its own time limit; a hard failure (rc not 0/1: fault, abort, time limit) ends the
# call there.  Outputs under gpurun_out/ (scratch; summaries worth keeping go to profiles/).
#   tests            pytest -m gpu (all GPU tests)          tests=EXPR   only -k EXPR
#   smoke            __graft_entry__.smoke()
#   bench            python bench.py (STEPS / WARMUP env, default 50 / 20)
#   trace            rocprofv3 --kernel-trace --stats over a short bench (prof_TAG/)
#   pmc              HBM traffic: FETCH_SIZE and WRITE_SIZE, one rocprofv3 run each (pmc_*_TAG/)
#   mfma             SQ_VALU_MFMA_BUSY_CYCLES & co. over a short bench (pmc_mfma_TAG/)
#   timeline         per-closure kernel timeline from the trace step's output
#   configs          tools/bench_configs.py (configs 1-5)
#   c4kin            tools/c4_kin.py: the fused config-4 Kin loop, ms per iteration + TorchSDF counters
#   c4trace          rocprofv3 --kernel-trace --stats over tools/c4_kin.py (prof_c4_TAG/)
#   sdfpmc           tools/pmc_sdf.sh: PMC passes over tools/sdf_child.py (the config-4 queries), sdf_tree_kernel
#   ab=SPEC,SPEC,..  interleaved bench A/B (R rounds, env R=3): SPEC = lib name ("base" = libcdx.so) with
#                    optional +VAR=VAL settings, e.g. ab=base,base+CDX_SCREEN_REPAIR=0
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
TAG=$1
shift
export TMPDIR=/tmp
STEPS=${STEPS:-50}
WARMUP=${WARMUP:-20}
stop_if_fault() { if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "GPU step failed hard (rc=$1): stopping"; exit "$1"; fi; }

for STEP in "$@"; do
  echo "== $STEP"; date
  case "$STEP" in
    tests|tests=*)
      K=()
      [ "$STEP" != tests ] && K=(-k "${STEP#tests=}")
      timeout -k 10 1000 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 240 --timeout-method thread \
        -rf "${K[@]}" > "$OUT/pytest_gpu_$TAG.log" 2>&1
      rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|ERROR" "$OUT/pytest_gpu_$TAG.log" | tail -12
      stop_if_fault $rc ;;
    smoke)
      timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke_$TAG.log" 2>&1
      rc=$?; echo "smoke rc=$rc"; tail -2 "$OUT/smoke_$TAG.log"; stop_if_fault $rc ;;
    bench)
      timeout -k 10 300 python bench.py --steps "$STEPS" --warmup "$WARMUP" > "$OUT/bench_$TAG.log" 2>&1
      rc=$?; echo "bench rc=$rc"; tail -c 3000 "$OUT/bench_$TAG.log"; stop_if_fault $rc ;;
    trace)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$TAG" -o run -- \
        python3 "$ROOT/bench.py" --steps 30 --warmup 20 --no-cpu-baseline --no-config4 > "$OUT/rocprof_$TAG.log" 2>&1
      rc=$?; echo "rocprof rc=$rc"; tail -2 "$OUT/rocprof_$TAG.log"; stop_if_fault $rc ;;
    pmc)
      for C in FETCH_SIZE WRITE_SIZE; do
        timeout -k 10 -s KILL 300 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmc_${C}_$TAG" -o run -- \
          python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-config4 > "$OUT/pmc_${C}_$TAG.log" 2>&1
        rc=$?; echo "pmc $C rc=$rc"; stop_if_fault $rc
      done ;;
    mfma)
      timeout -k 10 -s KILL 200 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_MFMA \
        SQ_WAVE_CYCLES --output-format csv -d "$OUT/pmc_mfma_$TAG" -o run -- \
        python3 "$ROOT/bench.py" --steps 3 --warmup 2 --no-cpu-baseline --no-config4 > "$OUT/pmc_mfma_$TAG.log" 2>&1
      rc=$?; echo "pmc mfma rc=$rc"; stop_if_fault $rc ;;
    timeline)
      python3 tools/closure_timeline.py "$OUT/prof_$TAG/run_kernel_trace.csv" > "$OUT/closure_timeline_$TAG.txt" 2>&1
      echo "timeline rc=$?"; tail -25 "$OUT/closure_timeline_$TAG.txt" ;;
    c4kin)
      timeout -k 10 300 python -u tools/c4_kin.py 20 3 > "$OUT/c4kin_$TAG.jsonl" 2> "$OUT/c4kin_$TAG.log"
      rc=$?; echo "c4kin rc=$rc"; cat "$OUT/c4kin_$TAG.jsonl"; tail -3 "$OUT/c4kin_$TAG.log"; stop_if_fault $rc ;;
    c4trace)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c4_$TAG" -o run -- \
        python3 "$ROOT/tools/c4_kin.py" 10 2 > "$OUT/rocprof_c4_$TAG.log" 2>&1
      rc=$?; echo "rocprof c4 rc=$rc"; tail -2 "$OUT/rocprof_c4_$TAG.log"; stop_if_fault $rc ;;
    sdfpmc)
      bash tools/pmc_sdf.sh "$TAG" > "$OUT/pmc_sdf_$TAG.txt" 2>&1
      rc=$?; echo "sdf pmc rc=$rc"; tail -40 "$OUT/pmc_sdf_$TAG.txt"; stop_if_fault $rc ;;
    sdfab=*)  # TorchSDF forward of the config-4 queries for each library: sdfab=base,name,... (libcdx_name.so)
      IFS=, read -r -a LIBS <<< "${STEP#sdfab=}"
      for r in $(seq 1 "${R:-2}"); do
        for L in "${LIBS[@]}"; do
          for K in around far; do
            if [ "$L" = base ]; then LP=$ROOT/compliancedex_amd/lib/libcdx.so; else LP=$ROOT/compliancedex_amd/lib/libcdx_$L.so; fi
            CDX_LIB=$LP timeout -k 10 120 python3 tools/sdf_child.py 6 $K > "$OUT/sdfab_run_$TAG.log" 2>&1
            rc=$?; [ $rc -ne 0 ] && { echo "$L rc=$rc"; tail -5 "$OUT/sdfab_run_$TAG.log"; exit $rc; }
            echo "{\"lib\": \"$L\", \"round\": $r, \"res\": $(grep '^{' "$OUT/sdfab_run_$TAG.log" | tail -1)}" | tee -a "$OUT/sdfab_$TAG.jsonl"
          done
        done
      done ;;
    c4ab=*)  # the fused config-4 Kin loop for each library: c4ab=base,name,...
      IFS=, read -r -a LIBS <<< "${STEP#c4ab=}"
      for r in $(seq 1 "${R:-2}"); do
        for L in "${LIBS[@]}"; do
          if [ "$L" = base ]; then LP=$ROOT/compliancedex_amd/lib/libcdx.so; else LP=$ROOT/compliancedex_amd/lib/libcdx_$L.so; fi
          CDX_LIB=$LP timeout -k 10 200 python3 tools/c4_kin.py 20 3 > "$OUT/c4ab_run_$TAG.log" 2>&1
          rc=$?; [ $rc -ne 0 ] && { echo "$L rc=$rc"; tail -5 "$OUT/c4ab_run_$TAG.log"; exit $rc; }
          grep '^{' "$OUT/c4ab_run_$TAG.log" | python3 -c "import json,sys; [print(json.dumps({'lib': '$L', 'round': $r, 'case': d['case'], 'min_ms': d['min_ms'], 'pairs_per_point': d['pairs_per_point']})) for d in map(json.loads, sys.stdin)]" | tee -a "$OUT/c4ab_$TAG.jsonl"
        done
      done ;;
    digest=*)  # config-2 closure output digests per library (bit-identity across builds): digest=base,name,...
      IFS=, read -r -a LIBS <<< "${STEP#digest=}"
      for L in "${LIBS[@]}"; do
        if [ "$L" = base ]; then LP=$ROOT/compliancedex_amd/lib/libcdx.so; else LP=$ROOT/compliancedex_amd/lib/libcdx_$L.so; fi
        CDX_LIB=$LP timeout -k 10 120 python3 tools/closure_digest.py 3 > "$OUT/digest_run_$TAG.log" 2>&1
        rc=$?; [ $rc -ne 0 ] && { echo "$L rc=$rc"; tail -5 "$OUT/digest_run_$TAG.log"; exit $rc; }
        grep '^{' "$OUT/digest_run_$TAG.log" | tail -1 | tee -a "$OUT/digest_$TAG.jsonl"
      done ;;
    configs)
      timeout -k 10 600 python -u tools/bench_configs.py --only "${CONFIGS:-c1,c2opt,c3,c4,c4loop,c5,fit}" > "$OUT/configs_$TAG.jsonl" 2> "$OUT/configs_$TAG.log"
      rc=$?; echo "configs rc=$rc"; tail -c 3000 "$OUT/configs_$TAG.jsonl"; stop_if_fault $rc ;;
    ab=*)
      IFS=, read -r -a SPECS <<< "${STEP#ab=}"
      for r in $(seq 1 "${R:-3}"); do
        for SPEC in "${SPECS[@]}"; do
          IFS=+ read -r L ENVS <<< "$SPEC"
          (
            for v in $(compgen -e | grep '^CDX_'); do unset "$v"; done  # each spec starts from the defaults
            if [ -n "$ENVS" ]; then for kv in ${ENVS//+/ }; do export "$kv"; done; fi
            if [ "$L" = base ]; then export CDX_LIB=$ROOT/compliancedex_amd/lib/libcdx.so
            else export CDX_LIB=$ROOT/compliancedex_amd/lib/libcdx_$L.so; fi
            timeout -k 10 200 python3 "$ROOT/bench.py" --steps "$STEPS" --warmup "$WARMUP" --no-cpu-baseline --no-config4 \
              > "$OUT/ab_run_$TAG.log" 2>&1
          )
          rc=$?; [ $rc -ne 0 ] && { echo "$SPEC rc=$rc"; tail -5 "$OUT/ab_run_$TAG.log"; exit $rc; }
          python3 -c "import json; d=json.loads([l for l in open('$OUT/ab_run_$TAG.log') if l.startswith('{')][-1]); print(json.dumps({'spec': '$SPEC', 'round': $r, 'ms_per_step': d['ms_per_step'], 'step_ms': d.get('step_ms'), 'stage_ms': d['stage_ms'], 'exact_rows': d.get('screen', {}).get('exact_rows')}))" | tee -a "$OUT/ab_$TAG.jsonl"
        done
      done ;;
    *) echo "unknown step $STEP"; exit 2 ;;
  esac
done
exit 0
