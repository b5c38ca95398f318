set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for rep in 1 2; do
for v in 32 4 2 1; do
  HDFS_CRC32C_SPEC_POOL=$v timeout -k 10 120 python tools/spec_phases.py gpurun_out/r5f_pool${v}_$rep.json > /dev/null 2> gpurun_out/r5f_pool${v}_$rep.err || exit $?
  python -c "
import json,statistics as st
d=json.load(open('gpurun_out/r5f_pool${v}_$rep.json'))
for k,v2 in d.items():
    rs=v2['runs']
    print('pool=$v rep=$rep', k, 'p4', st.median(r['p4_us'][0] for r in rs), 'p3max', st.median(r['p3_us'][2] for r in rs), 'wall', st.median(r['wall_us'] for r in rs))
"
done
done
