set -e
mkdir -p gpurun_out/cand
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/cand/pytest.log 2>&1
tail -1 gpurun_out/cand/pytest.log
python -u tools/ab_libs.py --libs raytracing-clj_amd/lib/ab_base.so raytracing-clj_amd/lib/librtclj.so --rounds 3 --out gpurun_out/cand/ab.jsonl
