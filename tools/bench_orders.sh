#!/bin/bash
# Bench the tiled-kernel schedules back to back on one box.
cd $GRAFT_REPO_ROOT
for o in ${ORDERS:-1 2 1 2}; do
  HDFS_CRC32C_TILE_ORDER=$o timeout -k 10 300 python bench.py --no-cpu --no-extra --steps 20 > /tmp/b.json || exit $?
  python -c "import json; d=json.load(open('/tmp/b.json')); print('order $o', d['value'], d['roofline']['frac'], d['parity']['mismatches'])"
done
