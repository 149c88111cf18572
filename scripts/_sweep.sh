set -u
cd $GRAFT_REPO_ROOT
for cfg in "SAY=4" "SAY=4 SY=8" "SH=16" "SAY=4 SH=16" "NONE=0"; do
  envs=""; for kv in $cfg; do envs="$envs SKR_HYP_$kv"; done
  tag=$(echo $cfg | tr ' =' '__')
  env $envs BENCH_TAG=$tag bash scripts/gpu_check.sh bench_env || exit $?
done
