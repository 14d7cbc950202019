# A/B timing of the headline under environment variants (one GPU call).
# Usage: bash scripts/gpu_ab.sh TAG "ENV1=a ENV2=b" "ENV1=c" ...
set -o pipefail
TAG=$1; shift
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
i=0
for v in "$@"; do
  i=$((i+1))
  env $v timeout -k 10 240 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extra > $O/ab_$i.json 2> $O/ab_$i.err || { echo "variant [$v] FAIL"; tail -20 $O/ab_$i.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$O/ab_$i.json')); print('[$v]', round(d['value']), 'tiles/s', round(d['ms_per_step'],3), 'ms', {k:round(v['ms'],3) for k,v in d.get('kernels',{}).items()} if isinstance(d.get('kernels'),dict) else '')"
done
