export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_check.sh r1c || exit 1
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/cal -o run --output-format csv -- tools/ubench/fetch_cal > gpurun_out/cal.log 2>&1 || { echo cal failed; exit 1; }
bash tools/pmc.sh r1c || exit 1
python tools/pmc_summary.py gpurun_out/pmc_r1c k_score_tiled3 1048576 5 48 gpurun_out/pmc_traffic.json > gpurun_out/pmc_r1c_summary.txt 2>&1
tail -3 gpurun_out/pmc_r1c_summary.txt
