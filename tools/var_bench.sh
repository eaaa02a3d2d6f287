set -e
for v in ${VARS:-base}; do
  if [ $v = base ]; then unset BK_LIB_PATH; else export BK_LIB_PATH=$GRAFT_REPO_ROOT/reinforcementlearning_blokus_amd/_lib/var_$v.so; fi
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 > gpurun_out/var_$v.json 2>gpurun_out/var_$v.err
  python -c "import json;d=json.load(open('gpurun_out/var_$v.json'));print('$v', round(d['value']/1e6,2), 'M sims/s', round(d['roofline']['kernel_ms'],3),'ms')"
done
