#!/bin/bash
# One-MI355X job runner (through gpurun, from the repo root): every job writes under
# gpurun_out/<tag>/, runs each GPU step under its own time limit and stops at the first GPU failure.
#
#   tools/gpu.sh verify  <tag> [quick]   GPU test suite, smoke(), bench.py; + ResNet benches unless quick
#   tools/gpu.sh persist <tag>           persistent flagship: numerics + phase timing, its tests, bench 20/200
#   tools/gpu.sh taxi    <tag>           fused taxi step: tests, phase stamps, 200-step bench, bench.py
#   tools/gpu.sh data    <tag>           50M-row Parquet -> HBM ingest, Titanic config 4, 2/4-rank rehearsals
#   tools/gpu.sh configs <tag>           every BASELINE config once (benchmarks/run.py) -> all.jsonl
#   tools/gpu.sh resnet  <tag>           CIFAR ResNet-20/56 + ResNet-50 B=64/256 benches and kernel tables
#   tools/gpu.sh prof    <tag>           rocprofv3 kernel table of bench.py (flagship only)
#   tools/gpu.sh pmc     <tag>           PMC passes over bench.py (one counter group per run)
#   tools/gpu.sh knobs   <tag> "ENV=.." ...   flagship bench.py --steps 20 per env setting ("" = default)
#   tools/gpu.sh debug   <tag>           kernel suites on the debug build (_hopsx_ops_dbg, HOPSX_DEBUG=1)
#   tools/gpu.sh ab      <tag> <reps> "<benchmarks/run.py args>" "ENV=.." ...   A/B of one benchmark config per
#                                        env setting ("" = default), <reps> rounds -> <tag>/ab.txt (the round-4
#                                        A/Bs in profiles/r4_*_ab.txt were run this way)
#   tools/gpu.sh tables  <tag>           rocprofv3 kernel tables of ResNet-20 (in-process) and ResNet-50 B=64
#   tools/gpu.sh dpsim   <tag>           persistent flagship DP exchange on distinct data (ExchangeSim, 2-process
#                                        peer, co-residency) + cooperative-launch A/B
#   tools/gpu.sh taxidp  <tag>           data-parallel v2 taxi step: 2/4/8 processes on one GPU, phases, tests
#   tools/gpu.sh numerics <tag>          ResNet-20 per-layer fp64 checks (runtime/layercheck.py) + P2P DP suites
#   tools/gpu.sh e1prof  <tag>           rocprofv3 kernel table of the E1 Keras fit (tools/e1_fit.py)
#   tools/gpu.sh convgemm <tag>          tools/bench_conv_gemm.py --torch at batch 64 and 8
set -o pipefail
job=${1:?job}; tag=${2:-$1}; shift 2
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
R=$(pwd)

fail() { tail -30 "$1"; exit 1; }
# pytest: 1 = an assertion failed (the GPU is fine, keep measuring); anything else stops the job
pyt() { local log=$1; shift; timeout -k 10 ${T:-300} python -u -m pytest ${PYX--x} -v --timeout 120 --timeout-method thread "$@" > $log 2>&1
        local rc=$?; tail -6 $log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc; }
bench() { local name=$1; shift; timeout -k 10 ${T:-300} python -u "$@" > $out/$name.json 2> $out/$name.err || fail $out/$name.err
          tail -1 $out/$name.json | cut -c1-400; }
ktable() { local d=$1 name=$2; shift 2
           timeout -k 10 ${T:-300} rocprofv3 --kernel-trace --stats -d $out/$d -o run -- python3 "$@" > $out/$d.log 2>&1 || fail $out/$d.log
           db=$(find $out/$d -name '*.db' | head -1); [ -n "$db" ] && python tools/profdb.py "$db" > $out/$name 2>&1
           f=$(find $out/$d -name '*kernel_stats.csv' | head -1); [ -n "$f" ] && cp "$f" $out/${name%.txt}_stats.csv
           rm -rf $out/$d; head -25 $out/$name; }

case $job in
verify)
  T=900 pyt $out/pytest_gpu.log tests -m gpu
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || fail $out/smoke.log
  bench bench bench.py --steps 20 --warmup 5
  [ "$1" = quick ] && exit 0
  bench cifar20 benchmarks/run.py cifar_resnet --depth 20 --batch 128 --steps 100 --warmup 10
  bench r50_b64 benchmarks/run.py resnet50 --batch 64 --steps 30 --warmup 5
  bench r50_b256 benchmarks/run.py resnet50 --batch 256 --steps 10 --warmup 3 ;;
persist)
  timeout -k 10 240 python -u tools/persist_check.py --steps 8 --timing 32 > $out/check.log 2>&1 || fail $out/check.log
  tail -40 $out/check.log
  pyt $out/pytest.log tests/test_persist_gpu.py
  bench bench20 bench.py --steps 20 --warmup 5 --no-taxi
  bench bench200 bench.py --steps 200 --warmup 20 --no-taxi ;;
taxi)
  pyt $out/pytest.log tests/test_taxi_v2_gpu.py tests/test_widedeep_fused_gpu.py tests/test_tfx_gpu.py
  timeout -k 10 180 python -u tools/taxi_phases.py > $out/phases.txt 2>&1 || fail $out/phases.txt
  cat $out/phases.txt
  bench taxi benchmarks/run.py taxi --steps 200 --warmup 20
  bench bench bench.py --steps 20 --warmup 5 ;;
data)
  T=400 bench ingest benchmarks/run.py titanic_ingest --rows 50000000
  bench titanic benchmarks/run.py titanic --rows 891000 --steps 300 --warmup 20
  for n in 2 4; do
    HOPSX_RANK_FAST_EXIT=0 PYTHONFAULTHANDLER=1 timeout -k 10 240 python -u bench.py --gpus $n --rehearse --steps 5 --warmup 2 --no-taxi > $out/rh$n.json 2> $out/rh$n.err
    rc=$?; echo "rehearsal $n ranks rc=$rc"; tail -3 $out/rh$n.json
    grep -n -i "terminate\|abort\|Fatal Python\|Segmentation" $out/rh$n.err | head -20
    [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
  done ;;
configs)
  : > $out/all.jsonl
  run() { timeout -k 10 300 python benchmarks/run.py "$@" 2>>$out/err.log | tail -1 >> $out/all.jsonl || fail $out/err.log; }
  run mnist_mirrored --steps 200 --warmup 20
  run taxi --steps 200 --warmup 20
  run taxi --steps 200 --warmup 20 --from-transform
  run titanic --steps 200 --warmup 20
  run cifar_resnet --depth 20 --batch 128 --steps 100 --warmup 10
  run cifar_resnet --depth 56 --batch 128 --steps 50 --warmup 10
  run resnet50 --batch 8 --steps 30 --warmup 5
  cut -c1-300 $out/all.jsonl ;;
resnet)
  bench cifar20 benchmarks/run.py cifar_resnet --depth 20 --batch 128 --steps 100 --warmup 10
  bench cifar56 benchmarks/run.py cifar_resnet --depth 56 --batch 128 --steps 50 --warmup 10
  bench r50_b64 benchmarks/run.py resnet50 --batch 64 --steps 30 --warmup 5
  bench r50_b256 benchmarks/run.py resnet50 --batch 256 --steps 10 --warmup 3
  ktable p20 r20_kernels.txt benchmarks/run.py cifar_resnet --depth 20 --batch 128 --steps 50 --warmup 10 --inline
  ktable p50 r50_b64_kernels.txt benchmarks/run.py resnet50 --batch 64 --steps 20 --warmup 5 ;;
prof)
  ktable pf flagship_kernels.txt bench.py --steps 200 --warmup 20 --no-taxi ;;
pmc)
  cd /tmp
  P="python3 $R/bench.py --steps 40 --warmup 10 --no-taxi"
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES -d "$R/$out/a" -o run --output-format csv -- $P > "$R/$out/a.log" 2>&1 && \
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES FETCH_SIZE -d "$R/$out/b" -o run --output-format csv -- $P > "$R/$out/b.log" 2>&1 && \
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES WRITE_SIZE -d "$R/$out/c" -o run --output-format csv -- $P > "$R/$out/c.log" 2>&1 ;;
debug)
  export HOPSX_DEBUG=1; T=600 pyt $out/pytest_debug.log tests/test_debug_checks_gpu.py tests/test_kernels_gpu.py tests/test_kernels_v2_gpu.py \
    tests/test_dgrad_par_gpu.py tests/test_wgrad_glds_gpu.py tests/test_bnstats_gpu.py tests/test_bn_fold_gpu.py \
    tests/test_models_gpu.py ;;
ab)
  reps=$1; args=$2; shift 2
  for rep in $(seq $reps); do for s in "" "$@"; do
    r=$(env $s timeout -k 10 300 python benchmarks/run.py $args 2>>$out/err.log | tail -1) || { echo "FAIL [$s]"; fail $out/err.log; }
    echo "[$s] $args -> $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a $out/ab.txt
  done; done ;;
taxipmc)
  # PMC passes over the taxi benchmark (one counter group per run): wave-cycles split, LDS, instruction mix
  cd /tmp
  P="python3 $R/benchmarks/run.py taxi --steps 64 --warmup 4"
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS -d "$R/$out/a" -o run --output-format csv -- $P > "$R/$out/a.log" 2>&1 && \
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_IFETCH -d "$R/$out/b" -o run --output-format csv -- $P > "$R/$out/b.log" 2>&1
  cd $R; python tools/pmcsum.py $out/a $out/b > $out/pmc.txt 2>&1; cat $out/pmc.txt | head -40 ;;
tables)
  ktable p20 r20_kernels.txt benchmarks/run.py cifar_resnet --depth 20 --batch 128 --steps 50 --warmup 10 --inline
  ktable p50 r50_b64_kernels.txt benchmarks/run.py resnet50 --batch 64 --steps 20 --warmup 5 ;;
taxidp)
  # the data-parallel v2 taxi step: 2/4/8 processes sharing the GPU (phase stamps + steps/s), its tests
  bash tools/taxi_dp_phases.sh $tag || exit 1
  pyt $out/pytest.log tests/test_taxi_dp_gpu.py tests/test_taxi_v2_gpu.py ;;
numerics)
  # per-layer (teacher-forced fp64) ResNet-20 numerics + the whole-step tests built on them; P2P DP suites
  T=900 PYX= pyt $out/layers.log tests/test_resnet_layers_gpu.py tests/test_bnstats_gpu.py tests/test_kernels_v2_gpu.py \
    tests/test_bn_dgrad_sums_gpu.py -s
  T=600 PYX= pyt $out/p2p.log tests/test_p2p_gpu.py -s; grep DPRESNET $out/p2p.log | cut -c1-600 ;;
e1prof)
  ktable pf e1_kernels.txt tools/e1_fit.py ;;
convgemm)
  for b in 64 8; do
    timeout -k 10 300 python -u tools/bench_conv_gemm.py --batch $b --torch > $out/convgemm_b$b.jsonl 2> $out/convgemm_b$b.err || fail $out/convgemm_b$b.err
  done ;;
dpsim)
  # the persistent flagship's data-parallel exchange on distinct per-rank data (ExchangeSim, cross-process
  # peer, co-residency), its loopback / one-GPU suites, and the cooperative-launch A/B on the bench
  T=600 pyt $out/pytest.log tests/test_persist_dp_sim_gpu.py tests/test_persist_dp_gpu.py tests/test_persist_gpu.py -s
  for s in "HOPSX_PERSIST_COOP=0" "HOPSX_PERSIST_COOP=1" "HOPSX_PERSIST_COOP=0" "HOPSX_PERSIST_COOP=1"; do
    r=$(env $s timeout -k 10 120 python bench.py --steps 200 --warmup 20 --no-taxi 2>>$out/err.log) || { echo "FAIL [$s]"; fail $out/err.log; }
    echo "[$s] $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')" | tee -a $out/ab.txt
  done ;;
knobs)
  for s in "$@"; do
    r=$(env $s timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-taxi 2>>$out/err.log) || { echo "FAIL [$s]"; fail $out/err.log; }
    echo "[$s] $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')" | tee -a $out/ab.txt
  done ;;
*) echo "unknown job $job"; exit 2 ;;
esac
exit 0
