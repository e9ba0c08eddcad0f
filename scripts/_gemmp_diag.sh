set -e
mkdir -p gpurun_out/gemmp_diag
for D in 0 3 4 0; do MADNN_GEMMP_DIAG=$D timeout -k 10 200 python -u bench/gemmp_epi_ab.py >> gpurun_out/gemmp_diag/ab.jsonl 2>gpurun_out/gemmp_diag/err_$D.log; done
cat gpurun_out/gemmp_diag/ab.jsonl
