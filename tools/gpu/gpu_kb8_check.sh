set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03b
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_ba_gpu.py tests/test_golden_ba.py -m gpu -x -q --timeout 120 --timeout-method thread -k "kb8 or golden or batch" > $OUT/pytest.log 2>&1 &&
timeout -k 10 200 python tools/pose_bench.py > $OUT/pose_bench.jsonl 2> $OUT/pose_bench.err
echo "exit=$?"
