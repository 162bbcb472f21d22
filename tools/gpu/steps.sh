#!/bin/bash
# One GPU call, named steps run in order; the first failing step ends the call (no GPU step after a
# fault, abort or time limit). Replaces the per-run rNN*.sh scripts of earlier rounds.
#   bash tools/gpu/steps.sh <tag> <step> [<step> ...]      -> gpurun_out/<tag>/
# steps:
#   race              tools/lds_race.py on the product library and, if built, libcomet_hip_nodrain.so
#   det2[:ENV=V,..]   two processes sharing the GPU, each running tools/determinism.py (3 training
#                     steps, outputs + gradients compared bit for bit); optional env for both
#   rec2[:ENV=V,..]   two processes at once, each running tools/op_record.py (first differing op
#                     output of three forward passes, with where it differs)
#   pair:<cmd+args>   python <cmd args> twice at once (words joined by '+')
#   noise:<cmd+args>  python <cmd args> beside a torch-only load process (tools/gpu_noise.py)
#   duo:<cmdA>@<cmdB> two different commands at once (words joined by '+')
#   ab:<VAR=V,..>     bench line A/B/A/B: default and with the environment
#   t:<pytest -k expr>  GPU tests selected by -k (one process)
#   f:<test path>     one GPU test file or node id
#   suite             the whole GPU suite (-m gpu)
#   smoke             __graft_entry__.smoke()
#   bench[:args]      python bench.py [args] -> bench*.json
#   prof              rocprofv3 kernel-trace statistics of the bench step
#   py:<cmd+args>     python <cmd args> alone (words joined by '+'; leading VAR=V words -> env)
#   pmcg:<M+N+K+act+dt+res>[@VAR=V]  FETCH_SIZE and WRITE_SIZE passes (one each) over tools/gemm_one.py
set -o pipefail
TAG=${1:?tag}
shift
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/$TAG
mkdir -p $O
n=0
fail() { echo "step failed ($1): $2"; exit 1; }
for s in "$@"; do
  n=$((n + 1))
  echo "== [$n] $s ($(date +%T))"
  case $s in
    race)
      timeout -k 10 300 python -u tools/lds_race.py 40 > $O/race_product.txt 2>&1 || fail $? "$s"
      cat $O/race_product.txt
      if [ -f comet-pose-estimation_amd/libcomet_hip_nodrain.so ]; then
        COMET_HIP_LIB=$PWD/comet-pose-estimation_amd/libcomet_hip_nodrain.so timeout -k 10 300 \
          python -u tools/lds_race.py 40 > $O/race_nodrain.txt 2>&1 || fail $? "$s nodrain"
        cat $O/race_nodrain.txt
      fi ;;
    det2|det2:*)
      envs=""
      [ "$s" != det2 ] && envs=$(echo ${s#det2:} | tr ',' ' ')
      arm=$(echo "${envs:-default}" | tr ' =' '_-')
      env $envs timeout -k 10 300 python -u tools/determinism.py 1 bf16 > $O/det2_${arm}_a.txt 2>&1 &
      pa=$!
      env $envs timeout -k 10 300 python -u tools/determinism.py 1 bf16 > $O/det2_${arm}_b.txt 2>&1
      rb=$?
      wait $pa
      ra=$?
      grep -h "keys differ\|out\." $O/det2_${arm}_a.txt $O/det2_${arm}_b.txt | head -20
      [ $ra -eq 0 ] && [ $rb -eq 0 ] || fail "$ra/$rb" "$s" ;;
    rec2|rec2:*)
      envs=""
      [ "$s" != rec2 ] && envs=$(echo ${s#rec2:} | tr ',' ' ')
      env $envs timeout -k 10 400 python -u tools/op_record.py bf16 > $O/rec2_a.txt 2>&1 &
      pa=$!
      env $envs timeout -k 10 400 python -u tools/op_record.py bf16 > $O/rec2_b.txt 2>&1
      rb=$?
      wait $pa
      ra=$?
      head -60 $O/rec2_a.txt
      [ $ra -eq 0 ] && [ $rb -eq 0 ] || fail "$ra/$rb" "$s" ;;
    pair:*)
      # pair:<script and args, words joined by '+'>: the same command twice at once
      cmd=$(echo ${s#pair:} | tr '+' ' ')
      tagp=$(echo ${s#pair:} | tr '+/.' '___')
      timeout -k 10 200 python -u $cmd > $O/${tagp}_a.txt 2>&1 &
      pa=$!
      timeout -k 10 200 python -u $cmd > $O/${tagp}_b.txt 2>&1
      rb=$?
      wait $pa
      ra=$?
      cat $O/${tagp}_a.txt $O/${tagp}_b.txt | grep -v amdgpu.ids
      [ $ra -eq 0 ] && [ $rb -eq 0 ] || fail "$ra/$rb" "$s" ;;
    noise:*)
      # noise:<cmd+args>: python <cmd args> beside tools/gpu_noise.py (torch GEMMs + copies, no
      # kernels of this library) in a second process
      cmd=$(echo ${s#noise:} | tr '+' ' ')
      tagp=$(echo ${s#noise:} | tr '+/.' '___')
      timeout -k 10 200 python -u tools/gpu_noise.py 75 > $O/${tagp}_noise.txt 2>&1 &
      pa=$!
      sleep 8
      timeout -k 10 200 python -u $cmd > $O/${tagp}_alone.txt 2>&1
      rb=$?
      wait $pa
      ra=$?
      cat $O/${tagp}_alone.txt $O/${tagp}_noise.txt | grep -v amdgpu.ids
      [ $ra -eq 0 ] && [ $rb -eq 0 ] || fail "$ra/$rb" "$s" ;;
    duo:*)
      # duo:<cmdA+args>@<cmdB+args>: two different commands at once (A's output is the one read)
      spec=${s#duo:}
      ca=$(echo ${spec%@*} | tr '+' ' ')
      cb=$(echo ${spec#*@} | tr '+' ' ')
      tagp=$(echo "$spec" | tr '+/.@' '____' | cut -c1-80)
      # leading VAR=VALUE words of a command go to its environment
      ea=""; while [[ $ca == *=* && ${ca%% *} == *=* ]]; do ea="$ea ${ca%% *}"; ca=${ca#* }; done
      eb=""; while [[ $cb == *=* && ${cb%% *} == *=* ]]; do eb="$eb ${cb%% *}"; cb=${cb#* }; done
      env $eb timeout -k 10 200 python -u $cb > $O/${tagp}_B.txt 2>&1 &
      pb=$!
      sleep 6
      env $ea timeout -k 10 200 python -u $ca > $O/${tagp}_A.txt 2>&1
      ra=$?
      wait $pb
      rb=$?
      cat $O/${tagp}_A.txt $O/${tagp}_B.txt | grep -v amdgpu.ids | grep -v "device re-read\|host copy"
      [ $ra -eq 0 ] && [ $rb -eq 0 ] || fail "$ra/$rb" "$s" ;;
    ab:*)
      # ab:<VAR=V,..>: bench line default / with the env / default / with the env (same box)
      envs=$(echo ${s#ab:} | tr ',' ' ')
      for arm in a1 b1 a2 b2; do
        e="X=1"; [[ $arm == b* ]] && e="$envs"
        env $e timeout -k 10 300 python bench.py --no-cpu-baseline > $O/ab_$arm.json 2> $O/ab_$arm.err || { tail $O/ab_$arm.err; fail $? "$s $arm"; }
        python -c "import json;d=json.loads(open('$O/ab_$arm.json').read().strip().splitlines()[-1]);print('$arm', '$e', d['value'], d['ms_per_step'])"
      done ;;
    t:*)
      timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests -k "${s#t:}" \
        > $O/tests_$n.log 2>&1 || { tail -30 $O/tests_$n.log; fail $? "$s"; }
      tail -3 $O/tests_$n.log ;;
    f:*)
      timeout -k 10 900 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread -m gpu "${s#f:}" \
        > $O/tests_$n.log 2>&1 || { tail -30 $O/tests_$n.log; fail $? "$s"; }
      tail -3 $O/tests_$n.log ;;
    suite)
      timeout -k 10 1000 python -u -m pytest -q -m gpu --timeout 300 --timeout-method thread tests \
        > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; fail $? "$s"; }
      tail -3 $O/gpu_tests.log ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || fail $? "$s"
      tail -3 $O/smoke.log ;;
    bench|bench:*)
      args=""
      [ "$s" != bench ] && args=$(echo ${s#bench:} | tr ',' ' ')
      out=$O/bench$(echo "$args" | tr -d ' -').json
      timeout -k 10 400 python bench.py $args > $out 2> $out.err || { tail $out.err; fail $? "$s"; }
      tail -c 600 $out; echo ;;
    prof)
      timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $O/prof -o run -- python bench.py --no-cpu-baseline \
        --steps 5 --warmup 2 > $O/bench_prof.json 2> $O/bench_prof.err || fail $? "$s" ;;
    py:*)
      cmd=$(echo ${s#py:} | tr '+' ' ')
      tagp=py${n}_$(echo ${s#py:} | tr '+/.=' '____' | rev | cut -c1-60 | rev)
      e=""; while [[ $cmd == *=* && ${cmd%% *} == *=* ]]; do e="$e ${cmd%% *}"; cmd=${cmd#* }; done
      env X=1 $e timeout -k 10 300 python -u $cmd > $O/$tagp.txt 2>&1 || { tail -20 $O/$tagp.txt; fail $? "$s"; }
      grep -v amdgpu.ids $O/$tagp.txt | tail -40 ;;
    pmcg:*)
      spec=${s#pmcg:}
      shp=$(echo ${spec%@*} | tr '+' ' ')
      e="X=1"; [[ $spec == *@* ]] && e=$(echo ${spec#*@} | tr ',' ' ')
      tagp=pmcg_$(echo "$spec" | tr '+@=,' '____')
      for c in FETCH_SIZE WRITE_SIZE; do
        env $e timeout -s KILL 90 rocprofv3 --pmc $c --kernel-trace --stats -f csv -d $O/$tagp/$c -o run -- python tools/gemm_one.py $shp 10 \
          > $O/${tagp}_$c.log 2>&1 || { tail $O/${tagp}_$c.log; fail $? "$s $c"; }
      done
      python tools/pmc_kernel.py $O/$tagp comet_gemm ;;
    *) fail 2 "unknown step $s" ;;
  esac
done
echo "all steps done"
