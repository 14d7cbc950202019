# Round-5 record: smoke, the bench line, and rocprofv3 kernel stats of the headline batch.
set -o pipefail
mkdir -p gpurun_out/r05zh
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r05zh/smoke.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > gpurun_out/r05zh/bench.log 2>&1 || exit 1
PBX_KSTREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05zh/prof -o run -- python3 scripts/prof_workload.py noise 5 > gpurun_out/r05zh/prof.log 2>&1 || exit 1
