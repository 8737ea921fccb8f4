set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac; return 0; }
step gemm timeout -k 10 300 python tools/gemm_bench.py > gpurun_out/gemm_bench.log 2>&1; grep "^{" gpurun_out/gemm_bench.log | python3 -c "
import sys, json
for l in sys.stdin:
    d=json.loads(l); print(d['M'],d['N'],d['K'], {k:v for k,v in d.items() if k.endswith('_ms')})"
exit 0
