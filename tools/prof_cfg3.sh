set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -m pytest tests/test_gpu_q16.py -m gpu -q -x > gpurun_out/q16b_tests.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_cfg3/trace -o run -- python3 tools/bench_configs.py --only cfg3 --repeat 1 > gpurun_out/prof_cfg3.json 2> gpurun_out/prof_cfg3.err
