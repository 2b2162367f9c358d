# query-file parse timing on the box's CPU share (host only)
mkdir -p gpurun_out
python3 -c "
import random
r=random.Random(1)
with open('/tmp/q1m.txt','w') as f:
    f.write('1000000\n')
    f.write(''.join('%d %d\n'%(r.randrange(1000000), r.randrange(1000000)) for _ in range(1000000)))
"
nproc > gpurun_out/r05ac_qtime.log; cat /sys/fs/cgroup/cpu.max >> gpurun_out/r05ac_qtime.log 2>&1
timeout 120 tools_scripts/bin/qtime /tmp/q1m.txt >> gpurun_out/r05ac_qtime.log 2>&1
timeout 120 tools_scripts/bin/qt2 /tmp/q1m.txt >> gpurun_out/r05ac_qtime.log 2>&1
cat gpurun_out/r05ac_qtime.log
