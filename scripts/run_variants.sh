cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/gpu_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
for v in 1 0; do
PGPU_SCAN=$v PGPU_TRACE=1 timeout -k 10 300 python -u bench.py --segments-per-gpu 200 --steps 3 --warmup 2 --no-cpu-baseline --no-bytes > gpurun_out/bench_trace_$v.log 2>&1 || { tail -5 gpurun_out/bench_trace_$v.log; exit 1; }
echo "scan=$v"; grep pgpu gpurun_out/bench_trace_$v.log | tail -3
PGPU_SCAN=$v timeout -k 10 300 python -u bench.py --segments-per-gpu 200 --steps 20 --warmup 3 --no-cpu-baseline --host-profile > gpurun_out/bench_$v.log 2>&1 || { tail -5 gpurun_out/bench_$v.log; exit 1; }
tail -1 gpurun_out/bench_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline'], d['host_profile_us'])"
done
