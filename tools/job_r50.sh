# ResNet-50: conv GEMM layer table vs PyTorch (fwd / dgrad / wgrad) at B=64 and B=8, the B=8 / B=64 benches,
# and a rocprofv3 kernel table of the B=8 step
set -o pipefail
o=gpurun_out/${1:-r5_r50}; mkdir -p $o
export TMPDIR=/tmp
for b in 64 8; do
  timeout -k 10 300 python -u tools/bench_conv_gemm.py --batch $b --torch > $o/convgemm_b$b.jsonl 2> $o/convgemm_b$b.err || { tail -20 $o/convgemm_b$b.err; exit 1; }
  tail -1 $o/convgemm_b$b.jsonl
done
for b in 8 64; do
  timeout -k 10 300 python -u benchmarks/run.py resnet50 --batch $b --steps 30 --warmup 5 > $o/r50_b$b.json 2> $o/r50_b$b.err || { tail -20 $o/r50_b$b.err; exit 1; }
  tail -1 $o/r50_b$b.json | cut -c1-400
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/pf8 -o run -- python3 benchmarks/run.py resnet50 --batch 8 --steps 20 --warmup 5 > $o/pf8.log 2>&1 || { tail -20 $o/pf8.log; exit 1; }
db=$(find $o/pf8 -name '*.db' | head -1); python tools/profdb.py "$db" "ResNet-50 B=8 (20 timed + warm-up steps)" > $o/r50_b8_kernels.txt 2>&1
rm -rf $o/pf8; head -32 $o/r50_b8_kernels.txt
