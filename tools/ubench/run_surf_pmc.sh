set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_surf
timeout -k 10 120 ./tools/ubench/valu_rates > gpurun_out/valu_rates2.txt 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU -f csv -d gpurun_out/pmc_surf/sq -o run -- python3 tools/bench_configs.py --only cfg5s --repeat 1 > gpurun_out/pmc_surf/sq.json 2> gpurun_out/pmc_surf/sq.err
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_WAVES -f csv -d gpurun_out/pmc_surf/grbm -o run -- python3 tools/bench_configs.py --only cfg5s --repeat 1 > gpurun_out/pmc_surf/grbm.json 2> gpurun_out/pmc_surf/grbm.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/pmc_surf/trace -o run -- python3 tools/bench_configs.py --only cfg5s --repeat 1 > gpurun_out/pmc_surf/trace.json 2> gpurun_out/pmc_surf/trace.err
python3 tools/pmc_table.py gpurun_out/pmc_surf > gpurun_out/pmc_surf/table.txt
