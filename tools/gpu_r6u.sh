set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6u
# (normal interpreter exit is the default since round 6)
for f in test_defer_gpu test_ingest_gpu test_multigpu_links test_rccl_loopback_gpu test_rccl_native_gpu; do
  timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/$f.py > gpurun_out/r6u/$f.log 2>&1
  rc=$?
  echo "$f rc=$rc" >> gpurun_out/r6u/rc.txt
  [ $rc -eq 0 ] || exit $rc
done
