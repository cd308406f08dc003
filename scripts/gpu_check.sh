set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
mkdir -p gpurun_out
rocm-smi --showproductname > gpurun_out/smi.txt 2>&1 || true
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -m gpu -x -q > gpurun_out/pytest_kernels.log 2>&1 ; echo "kernels rc=$?" >> gpurun_out/status.txt
tail -5 gpurun_out/pytest_kernels.log
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -m gpu -q --maxfail=15 > gpurun_out/pytest_parity.log 2>&1 ; echo "parity rc=$?" >> gpurun_out/status.txt
tail -25 gpurun_out/pytest_parity.log
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/bench1.json 2> gpurun_out/bench1.err ; echo "bench rc=$?" >> gpurun_out/status.txt
cat gpurun_out/bench1.json; tail -3 gpurun_out/bench1.err
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --variant 2 > gpurun_out/bench1_v2.json 2>> gpurun_out/bench1.err ; echo "bench v2 rc=$?" >> gpurun_out/status.txt
cat gpurun_out/bench1_v2.json
cat gpurun_out/status.txt
