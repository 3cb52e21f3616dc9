mkdir -p gpurun_out/r05t
for v in hoisted entry; do
  if [ $v = entry ]; then L=graph-distillation-for-recommendation_amd/gdd/lib/libgdd_stopentry.so; else L=graph-distillation-for-recommendation_amd/gdd/lib/libgdd.so; fi
  timeout -k 10 300 env GDD_LIB_PATH=$L rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05t/$v -o bench -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extra > gpurun_out/r05t/$v.log 2>&1 || exit 1
  echo "== $v"
  for k in k_mb_assign k_minibatch_update k_mb_reassign k_kpp1_dm2; do python3 tools/kernel_durations.py gpurun_out/r05t/$v/bench_kernel_trace.csv $k 3; done
done
