#!/usr/bin/env bash
# Counter passes over the general GEMM (square bf16 and the fp32 dense forward shape).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
O=gpurun_out/gemm_pmc
mkdir -p $O
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES"
P2="SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD"
for shape in "4096 4096 4096 bf16" "65536 784 128 fp32"; do
  tag=$(echo $shape | tr ' ' '_')
  timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d $O/kt_$tag -o kt -- python3 tools/probes/gemm_one.py $shape > $O/kt_$tag.log 2>&1 || exit $?
  timeout -s KILL 90 rocprofv3 --pmc $P1 -d $O/p1_$tag -o p1 -- python3 tools/probes/gemm_one.py $shape > $O/p1_$tag.log 2>&1 || exit $?
  timeout -s KILL 90 rocprofv3 --pmc $P2 -d $O/p2_$tag -o p2 -- python3 tools/probes/gemm_one.py $shape > $O/p2_$tag.log 2>&1 || exit $?
done
echo done
