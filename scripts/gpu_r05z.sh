# Round-5 regression hunt: the headline batch (prof_workload noise) on the round-3 final tree,
# round-4 trees before / after the match carry, the round-4 final tree and the current tree,
# alternating on one box.
set -o pipefail
mkdir -p gpurun_out/r05z
for i in 1 2 3; do
  for t in _ab/cef8494 _ab/40739cc _ab/b013c52 _ab/0486e88 .; do
    echo "== $t"
    (cd $t && timeout -k 10 200 python -u scripts/prof_workload.py noise 4 | tail -n 3) || exit 1
  done
done > gpurun_out/r05z/ab.log 2>&1
