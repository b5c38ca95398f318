#!/bin/bash
# Mailbox compute-phase experiments (diagnostic build): phase traces with
# parts of the per-lane work switched off (see mailbox_kernel's exp flags).
set -e
for e in 0 1 2 4 7; do
  HDFS_CRC32C_SMALL_TRACE=1 HDFS_CRC32C_MB_EXP=$e timeout -k 10 60 python -u tools/mailbox_trace.py > gpurun_out/mbexp_$e.log 2>&1
done
