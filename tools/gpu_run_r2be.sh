source tools/gpu_steps.sh
for k in 1 2; do
step t16 300 python -u tools/train_bench.py --no-cpu-baseline --steps 30 > gpurun_out/tr16.json 2>&1
echo "16-lane: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/tr16.json)"
APN_CELL_BOUND16_MAX=0 step t1 300 python -u tools/train_bench.py --no-cpu-baseline --steps 30 > gpurun_out/tr1.json 2>&1
echo "1-lane: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/tr1.json)"
done
