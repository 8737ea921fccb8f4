set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac; return 0; }
step p1 timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS -d gpurun_out/prof/p1 -o p1 --output-format csv -- python tools/gemm_prof.py > gpurun_out/prof/p1.log 2>&1
step p2 timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_VMEM SQ_INSTS_MFMA -d gpurun_out/prof/p2 -o p2 --output-format csv -- python tools/gemm_prof.py > gpurun_out/prof/p2.log 2>&1
find gpurun_out/prof -name "*.csv" | head
exit 0
