# Round-5 diagnostic: k_lz77 walk steps and repair rounds per segment (PBX_PHASE_PROFILE, phase
# report's "7:" = mean walk steps of a workgroup + 2^20 x wave 0's repair rounds) on G_NOISE,
# G_FAKE, and G_FAKE with the Up / adaptive filters.
set -o pipefail
mkdir -p gpurun_out/r05zp
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for F in 0 2 5; do for G in noise fake; do echo "== filter $F $G"; PBX_PNG_FILTER=$F PBX_PHASE_PROFILE=1 timeout -k 10 120 python -u scripts/phase_profile.py $G 1024 2>&1 || exit 1; done; done > gpurun_out/r05zp/walk.log 2>&1 || exit 1
V=$PWD/omero-ms-pixel-buffer_amd/lib
for F in 0 5; do echo "== walk-prof filter $F fake"; PBX_LIB=$V/var_wp/libpbx.so PBX_PNG_FILTER=$F PBX_PHASE_PROFILE=1 timeout -k 10 120 python -u scripts/phase_profile.py fake 1024 2>&1 || exit 1; done >> gpurun_out/r05zp/walk.log 2>&1 || exit 1
