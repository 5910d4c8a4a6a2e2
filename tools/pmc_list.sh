# Two PMC passes over the C4 (List) decode: per-kernel SQ counters.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU --output-format csv -d gpurun_out/pmcl1 -o p -- python3 tools/c4bench.py ${ROWS:-10000000} > gpurun_out/pmcl1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LEVEL_WAVES --output-format csv -d gpurun_out/pmcl2 -o p -- python3 tools/c4bench.py ${ROWS:-10000000} > gpurun_out/pmcl2.log 2>&1 || exit 1
ls gpurun_out/pmcl1 gpurun_out/pmcl2
