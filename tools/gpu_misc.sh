set -e
mkdir -p gpurun_out/cmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/cmp/pytest.log 2>&1
tail -1 gpurun_out/cmp/pytest.log
python -u tools/ab_libs.py --libs raytracing-clj_amd/lib/ab_base.so raytracing-clj_amd/lib/librtclj.so --rounds 3 --out gpurun_out/cmp/ab.jsonl
