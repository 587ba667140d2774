set -e
mkdir -p gpurun_out/pool
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pool/pytest.log 2>&1
tail -1 gpurun_out/pool/pytest.log
for wl in c1 c2; do
  timeout -k 10 300 python -u bench.py --workload $wl --steps 3 --warmup 1 --cpu-baseline off > gpurun_out/pool/$wl.json 2> gpurun_out/pool/$wl.err
  python -c "import json; d=json.load(open('gpurun_out/pool/$wl.json')); print('$wl', round(d['value']), round(d['kernel_ms_avg'],2), json.dumps(d['bvh_per_segment']['per_wave_iter']))"
done
