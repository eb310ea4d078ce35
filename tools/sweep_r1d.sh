set -e
B="timeout -k 10 240 python bench.py --no-cpu-baseline"
$B --steps 10 --warmup 3 > gpurun_out/s_default.json
$B --mode final --height 320 --width 320 --steps 20 --warmup 5 > gpurun_out/s_final320.json
DGVCC_SPLITK=0 $B --mode final --height 320 --width 320 --steps 20 --warmup 5 > gpurun_out/s_final320_nosplit.json
$B --mode final --steps 8 --warmup 3 > gpurun_out/s_final.json
