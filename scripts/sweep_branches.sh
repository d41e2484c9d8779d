# HDCE side-branch plans (FlagshipConfig.hdce_branches / fc_adam_grid), alternating with the default
set -o pipefail
mkdir -p gpurun_out
for v in "x 0" "a 0" "a 128" "a 64" "x 0" "a 0" "wa 0" "w 0"; do set -- $v; br=${1/x/}
  timeout -k 10 200 python bench.py --steps 300 --warmup 10 --hdce-branches=$br --fc-adam-grid $2 > gpurun_out/b.log 2>&1 || { tail -20 gpurun_out/b.log; exit 1; }
  echo "branches=$1 grid=$2 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/b.log)"
done
