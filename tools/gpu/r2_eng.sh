set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for cfg in "raftstereo-sceneflow 8 10" "raftstereo-sceneflow 1 20" "raftstereo-realtime 1 20" "crestereo-iter10 1 20"; do set -- $cfg
  SA_PLAN_CACHE=gpurun_out/plan_${1}_b$2.txt timeout -k 10 200 python -u tools/run_engine.py --model $1 --batch $2 --frames $3 2>&1 | grep -v amdgpu.ids | tail -n 1 || exit 1
done
