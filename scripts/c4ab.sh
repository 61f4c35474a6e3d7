# C4 star-tree A/B: K6 workgroup counts (PGPU_STAR_WGS) and the scan path
for cfg in "X=0" "PGPU_STAR_WGS=128" "PGPU_STAR_WGS=512"; do
  env $cfg timeout -k 10 200 python -u bench.py --workload c4 --segments-per-gpu 64 --steps 20 --warmup 3 --no-pmc --no-cpu-baseline --host-profile > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$cfg', d['ms_per_step'], r.get('kernel_us'))"
done
