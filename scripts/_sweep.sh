set -u
cd $GRAFT_REPO_ROOT
for cfg in "SM=4" "SAM=16" "SH=64" "SY=8" "SAY=16" "SM=4 SAM=16"; do
  envs=""; for kv in $cfg; do envs="$envs SKR_HYP_$kv"; done
  tag=$(echo $cfg | tr ' =' '__')
  env $envs BENCH_TAG=$tag bash scripts/gpu_check.sh bench_env || exit $?
done
