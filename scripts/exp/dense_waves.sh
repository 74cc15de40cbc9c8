#!/bin/bash
# dense replay throughput vs waves in flight (config 3 shape, T=16384, L=87)
cd /root/repo
for g in 128 256 512 1024; do
  echo "grid $g"
  FSTAMD_DENSE_GRID=$g FSTAMD_DENSE_LPT=0 FSTAMD_DENSE_BUCKETS=1 timeout -k 10 200 python -u scripts/config3_scaling.py --ts 16384 --n 1024 --len 87 --cpu-max-t 0 || exit $?
done
