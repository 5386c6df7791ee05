# One parametrised GPU-box runner (replaces the per-session one-shot scripts).
#
#   bash tools/gpu.sh <tag> <step> [<step> ...]
#
# Every step runs under its own time limit, writes under gpurun_out/<tag>_*,
# and the first failing step ends the call (no GPU work after a fault).
# Steps:
#   tests            python -m pytest tests -m gpu (all)       -> <tag>_gpu_tests.log
#   tests:<expr>     the same with -k <expr>
#   smoke            __graft_entry__.smoke()                    -> <tag>_smoke.log
#   bench            python bench.py (default protocol)         -> <tag>_bench.json
#   prof             tools/profile_round.sh <tag> (kernel stats, FETCH/WRITE, MFMA busy)
#   inf              cfg5 at its stated config: --images 8192, fp32 and bf16
#                                                               -> <tag>_inference_cfg5_{fp32,bf16}.json
#   cfg2             tools/bench_cfg2.py                        -> <tag>_cfg2.jsonl
#   conv3r[:ARGS]    tools/ab_conv3r.py ARGS (comma lists; ';' separates switches)
#                                                               -> <tag>_conv3r.jsonl
#   abstep:NAME=a,b  graph-step A/B of one switch, alternating, 3 rounds
#                                                               -> <tag>_abstep.txt
#   ablibs:PATH      graph-step A/B of this build vs another .so -> <tag>_ablibs.txt
#   abconv:PATH      per-layer conv3r A/B of this build vs another .so -> <tag>_abconv.txt
#   ablayers:PATH[;SET] per-layer times + output SHA-1 of this build vs another .so
#                    (tools/layer_times.py SET = wgrad / conv3r) -> <tag>_ablayers_<SET>.txt
#   gtrace           rocprofv3 kernel trace of the graph-replayed bench -> <tag>_graph_trace.json
#   py:SCRIPT[;ARGS] python SCRIPT ARGS                         -> <tag>_py.log
set -o pipefail
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
O=gpurun_out/$TAG
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"

run_step() {
  local s=$1 arg=""
  case "$s" in *:*) arg=${s#*:}; s=${s%%:*};; esac
  echo "== $TAG $s $arg $(date +%T)"
  case "$s" in
    tests)
      if [ -n "$arg" ]; then
        timeout -k 10 1000 $T tests -m gpu -k "$arg" > ${O}_gpu_tests.log 2>&1
      else
        timeout -k 10 1000 $T tests -m gpu > ${O}_gpu_tests.log 2>&1
      fi
      local rc=$?; tail -3 ${O}_gpu_tests.log; return $rc ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > ${O}_smoke.log 2>&1
      local rc=$?; tail -2 ${O}_smoke.log; return $rc ;;
    bench)
      timeout -k 10 400 python bench.py > ${O}_bench.json 2> ${O}_bench.err
      local rc=$?; head -c 600 ${O}_bench.json; echo; return $rc ;;
    prof)
      timeout -k 10 1000 bash tools/profile_round.sh $TAG > ${O}_prof.log 2>&1
      local rc=$?; tail -5 ${O}_prof.log; return $rc ;;
    inf)
      timeout -k 10 400 python tools/bench_inference.py --images 8192 --dtype fp32 \
        > ${O}_inference_cfg5_fp32.json 2> ${O}_inf_fp32.err || return 1
      cat ${O}_inference_cfg5_fp32.json
      timeout -k 10 400 python tools/bench_inference.py --images 8192 --dtype bf16 \
        > ${O}_inference_cfg5_bf16.json 2> ${O}_inf_bf16.err || return 1
      cat ${O}_inference_cfg5_bf16.json ;;
    cfg2)
      timeout -k 10 400 python tools/bench_cfg2.py > ${O}_cfg2.jsonl 2> ${O}_cfg2.err
      local rc=$?; cat ${O}_cfg2.jsonl; return $rc ;;
    conv3r)
      timeout -k 10 600 python -u tools/ab_conv3r.py ${arg//;/ } > ${O}_conv3r.jsonl 2> ${O}_conv3r.err
      local rc=$?; tail -1 ${O}_conv3r.jsonl; return $rc ;;
    abstep)
      local name=${arg%%=*} vals=${arg#*=}
      for i in 1 2 3; do
        for v in ${vals//,/ }; do
          env $name=$v timeout -k 10 150 python bench.py --no-cpu-baseline --no-probe --steps 30 \
            > ${O}_ab.log 2>&1 || return 1
          tail -1 ${O}_ab.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$name=$v', d['value'], d['ms_per_step'])" >> ${O}_abstep.txt
        done
      done
      cat ${O}_abstep.txt ;;
    ablibs)
      for i in 1 2 3; do
        for L in cur other; do
          if [ $L = other ]; then export RR_LIB_PATH=$arg; else unset RR_LIB_PATH; fi
          timeout -k 10 150 python bench.py --no-cpu-baseline --no-probe --steps 30 > ${O}_ab.log 2>&1 || return 1
          tail -1 ${O}_ab.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$L', d['value'], d['ms_per_step'])" >> ${O}_ablibs.txt
        done
      done
      unset RR_LIB_PATH
      cat ${O}_ablibs.txt ;;
    abinf)
      # cfg5 bf16 inference of this build vs another .so, alternating
      # processes, 3 rounds (images/s, restore / judge ms per 1k images)
      for i in 1 2 3; do
        for L in cur other; do
          if [ $L = other ]; then export RR_LIB_PATH=$arg; else unset RR_LIB_PATH; fi
          timeout -k 10 300 python tools/bench_inference.py --images 4096 --dtype bf16 > ${O}_abinf.log 2>&1 || { unset RR_LIB_PATH; return 1; }
          tail -1 ${O}_abinf.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); s=d['stage_ms_per_1k_images']; print('$L', d['images_per_sec'], s['restore'], s['judge'], d['roofline']['restore']['frac'])" >> ${O}_abinf.txt
        done
      done
      unset RR_LIB_PATH
      cat ${O}_abinf.txt ;;
    abinfenv)
      # cfg5 bf16 inference per value of an environment switch, alternating,
      # 3 rounds: abinfenv:RR_PATH=conv3r_segwg=4,conv3r_segwg=8
      local name=${arg%%=*} vals=${arg#*=}
      for i in 1 2 3; do
        for v in ${vals//,/ }; do
          env $name=$v timeout -k 10 300 python tools/bench_inference.py --images 4096 --dtype bf16 > ${O}_abinf.log 2>&1 || return 1
          tail -1 ${O}_abinf.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); s=d['stage_ms_per_1k_images']; print('$name=$v', d['images_per_sec'], s['restore'], s['judge'], d['roofline']['restore']['frac'])" >> ${O}_abinfenv.txt
        done
      done
      cat ${O}_abinfenv.txt ;;
    abconv)
      # per-layer conv3r A/B of this build vs another .so (cfg3 and the 224
      # set), alternating processes, 3 rounds
      for i in 1 2 3; do
        for L in cur other; do
          for S in cfg3 224; do
            if [ $L = other ]; then export RR_LIB_PATH=$arg; else unset RR_LIB_PATH; fi
            if [ $S = 224 ]; then export SET=224; else unset SET; fi
            timeout -k 10 150 python -u tools/ab_conv3r.py > ${O}_abconv.log 2>&1 || return 1
            echo "$L $S $(tail -1 ${O}_abconv.log)" >> ${O}_abconv.txt
          done
        done
      done
      unset RR_LIB_PATH SET
      cat ${O}_abconv.txt ;;
    ablayers)
      # per-layer times + output SHA-1 (tools/layer_times.py SET) of this build
      # vs another .so, alternating processes, 3 rounds
      local other=${arg%%;*} set=${arg#*;}
      [ "$set" = "$arg" ] && set=wgrad
      for i in 1 2 3; do
        for L in cur other; do
          if [ $L = other ]; then export RR_LIB_PATH=$other; else unset RR_LIB_PATH; fi
          timeout -k 10 200 python -u tools/layer_times.py $set > ${O}_ablayers.log 2>&1 || { unset RR_LIB_PATH; return 1; }
          sed "s/^/$L $i /" ${O}_ablayers.log >> ${O}_ablayers_${set}.txt
        done
      done
      unset RR_LIB_PATH
      grep total_ms ${O}_ablayers_${set}.txt ;;
    gtrace)
      # rocprofv3 kernel trace of the HIP-graph replays of the driver's bench
      # command; tools/graph_trace.py: kernel sum vs wall per step
      rm -rf ${O}_gt
      timeout -k 10 300 rocprofv3 --kernel-trace -d ${O}_gt -o gt -- python bench.py --gpus 1 \
        --steps 20 --warmup 5 --no-cpu-baseline --no-probe > ${O}_gtrace_bench.json 2> ${O}_gtrace.err || return 1
      local db=$(find ${O}_gt -name "*.db" | head -1)
      python tools/graph_trace.py "$db" ${O}_graph_trace.json 20 ;;
    py)
      local script=${arg%%;*} rest=""
      [ "$script" != "$arg" ] && rest=${arg#*;}
      timeout -k 10 600 python -u $script ${rest//;/ } > ${O}_py.log 2>&1
      local rc=$?; tail -20 ${O}_py.log; return $rc ;;
    *) echo "unknown step $s"; return 2 ;;
  esac
}

for step in "$@"; do
  run_step "$step" || { echo "step $step failed rc=$?"; exit 1; }
done
echo "== $TAG done $(date +%T)"
