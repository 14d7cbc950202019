# Round-5 record (final code): the -m gpu suite, smoke, the bench line, rocprofv3 kernel stats
# of the headline batch on one kernel stream.
set -o pipefail
mkdir -p gpurun_out/r05zy
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/r05zy/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r05zy/smoke.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > gpurun_out/r05zy/bench.log 2>&1 || exit 1
PBX_KSTREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05zy/prof -o run -- python3 scripts/prof_workload.py noise 5 > gpurun_out/r05zy/prof.log 2>&1 || exit 1
