set -u
cd $GRAFT_REPO_ROOT
for cfg in "SAM=4" "SAY=4" "SAM=4 SAY=4" "SH=16" "SY=2" "SAM=2"; do
  envs=""; for kv in $cfg; do envs="$envs SKR_HYP_$kv"; done
  tag=$(echo $cfg | tr ' =' '__')
  env $envs BENCH_TAG=$tag bash scripts/gpu_check.sh bench_env || exit $?
done
