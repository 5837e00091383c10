cd "$GRAFT_REPO_ROOT" || exit 1
# Refresh the non-default config numbers of DESIGN.md §5/§6 (C5 arm shape, C4 genome, 10k TSV end to end).
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --n0 24300 --steps 3 --warmup 1 --no-cpu-baseline --throughput-streams 0 > gpurun_out/c5.log 2>&1
rc=$?; echo "c5 rc=$rc"; [ $rc -eq 0 ] || exit $rc
tail -1 gpurun_out/c5.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['stages_ms'], d['roofline']['classes']['coniss'])"
timeout -k 10 300 python tools/genome_bench.py > gpurun_out/c4.log 2>&1
rc=$?; echo "c4 rc=$rc"; tail -5 gpurun_out/c4.log
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --throughput-streams 0 --e2e-tsv 10000 > gpurun_out/tsv.log 2>&1
rc=$?; echo "tsv rc=$rc"; tail -1 gpurun_out/tsv.log | cut -c1-300; grep -o '"e2e[^}]*}' gpurun_out/tsv.log | head -2
exit $rc
