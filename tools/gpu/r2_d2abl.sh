# direct conv v2 statistics-cost ablations (SA_DIRECT2_ABL), fr8 / fnet
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for abl in 0 1 2 3; do SA_DIRECT2_ABL=$abl timeout -k 10 100 python -u tools/conv_bench.py --iters 20 --shapes fr8,fnet --cfgs=23 --stats 16 2>&1 | grep -v amdgpu.ids | sed "s/^/stats abl$abl /" || exit 1; done > gpurun_out/d2abl.log
for abl in 0 4; do SA_DIRECT2_ABL=$abl timeout -k 10 100 python -u tools/conv_bench.py --iters 20 --shapes fr8,fnet --cfgs=23 2>&1 | grep -v amdgpu.ids | sed "s/^/nostats abl$abl /" || exit 1; done >> gpurun_out/d2abl.log
cat gpurun_out/d2abl.log
