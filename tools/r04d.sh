#!/bin/bash
# round-4 check d: GPU tests of the exact mean correction, bench + profile,
# then the 16-bit vs 32-bit decision comparison
bash tools/r04_check.sh r04d tests/test_gpu_meancorr.py tests/test_gpu_families.py tests/test_gpu_devices.py || exit $?
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 600 python -u tools/q16_parity.py cfg2 n3k n8k n12k cfg4 > gpurun_out/r04d/q16_parity.jsonl 2> gpurun_out/r04d/q16_parity.err || exit $?
cat gpurun_out/r04d/q16_parity.jsonl
