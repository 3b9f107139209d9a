cd "${GRAFT_REPO_ROOT}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5n; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "group or dist or bench" > $O/pytest_group.txt 2>&1
rc=$?; tail -n 3 $O/pytest_group.txt; [ $rc -eq 0 ] || exit $rc
TAG=r5n/g REPEATS=2 bash tools/gpu_r5_gather.sh
