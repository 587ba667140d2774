set -e
mkdir -p gpurun_out/c4occ
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/c4occ/pytest.log 2>&1
tail -1 gpurun_out/c4occ/pytest.log
python -u tools/ab_libs.py --libs raytracing-clj_amd/lib/ab_base.so raytracing-clj_amd/lib/librtclj.so --rounds 3 --out gpurun_out/c4occ/ab_c1.jsonl
python -u tools/ab_libs.py --libs raytracing-clj_amd/lib/ab_base.so raytracing-clj_amd/lib/librtclj.so --rounds 2 --steps 1 --out gpurun_out/c4occ/ab_c4.jsonl -- --workload c4 --spp 200
