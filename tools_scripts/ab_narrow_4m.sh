set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out
timeout -k 10 400 python3 -u -m pytest $R/tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests_ad.log 2>&1
echo tests-done; tail -2 $O/gpu_tests_ad.log
B="python3 -u $R/bench.py --no-pmc --no-cpu --steps 3"
timeout -k 10 300 $B > $O/ad_1m.json 2> $O/ad_1m.err
timeout -k 10 600 $B --width 2000 > $O/ad_4m.json 2> $O/ad_4m.err
CPD_NARROW=0 timeout -k 10 300 $B --width 2000 > $O/ad_4m_wide.json 2> $O/ad_4m_wide.err
for f in ad_1m ad_4m ad_4m_wide; do python3 -c "
import json;d=json.load(open('$O/$f.json'));print('$f',d['value'],d['config']['rows_per_step_per_gpu'],d['narrow_rows'],{k:round(v['ms']/3,1) for k,v in d['kernels'].items()})"; done
