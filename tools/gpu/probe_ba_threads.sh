#!/bin/bash
# BA host-thread / batch-size probe (one gpurun call): LBA split of host phases vs device steps
# (OSG_LBA_PROFILE=1), then bench's local_ba / global_ba lines at a few (batch, threads) settings.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-p2}
mkdir -p $O
OSG_LBA_PROFILE=1 KT=1 TS=1,8 BS=64 timeout -k 10 200 python -u tools/lba_batch_bench.py > $O/lba_prof.txt 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu --no-stream --only local_ba --lba-threads 8 --ba-batch 128 > $O/lba_b128.json 2> $O/lba_b128.err &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu --no-stream --only local_ba --lba-threads 12 --ba-batch 96 > $O/lba_b96t12.json 2> $O/lba_b96t12.err &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu --no-stream --only global_ba --no-gba-map --gba-batch 16 --gba-threads 8 > $O/gba_16x8.json 2> $O/gba_16x8.err
echo "exit=$?"
