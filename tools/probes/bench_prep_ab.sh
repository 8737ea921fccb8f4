set -o pipefail
for arm in 0 54272 0 54272; do
  timeout -k 10 300 python -c "import sys; sys.argv=['bench.py']; import lumen_amd.ops as o; o._PREP_BAND_LDS=$arm; import runpy; runpy.run_path('bench.py', run_name='__main__')" > gpurun_out/bab_$arm.log 2>&1 || { echo "arm $arm failed"; tail -5 gpurun_out/bab_$arm.log; exit 1; }
  echo "arm=$arm $(grep '^{' gpurun_out/bab_$arm.log | cut -c1-110)"
done
