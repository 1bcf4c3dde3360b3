set -e
P="python tools/gemm_probe.py --impl 2 3 --iters 10"
$P --layout nt --M 32768 --N 4096 --K 768 --check --blas
$P --layout nt --M 32768 --N 2304 --K 768 --check
$P --layout nt --M 32768 --N 768 --K 768 --check --blas
$P --layout nt --M 32768 --N 768 --K 2048 --check --blas
$P --layout nt --M 32768 --N 50304 --K 768 --blas
$P --layout nt --M 32768 --N 4096 --K 3072 --check
$P --layout nn --M 32768 --N 768 --K 4096 --check --blas
$P --layout nn --M 32768 --N 768 --K 2048 --check --blas
$P --layout nn --M 32768 --N 4096 --K 768 --check --blas
$P --layout tn --M 32768 --N 4096 --K 768 --check --blas
$P --layout tn --M 32768 --N 768 --K 768 --check --blas
$P --layout nt --M 1000 --N 392 --K 200 --check
$P --layout tn --M 1000 --N 392 --K 200 --check
