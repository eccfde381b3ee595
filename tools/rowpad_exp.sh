for rp in 1 0 2; do
  LORA_MI355X_ROWPAD=$rp timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/rp_$rp.log 2>&1 || exit 1
done
