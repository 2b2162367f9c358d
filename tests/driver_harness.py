"""Local restatement of the reference head-node driver (process_query.py).

The reference reaches workers with `ssh host 'bash -s' < script`
(process_query.py:66-79).  The GPU box has no sshd, so this harness runs the
byte-identical script with `bash -s` locally.  Everything else follows the
reference line by line; tests/golden/driver_fixtures.json (captured from the
reference itself by tests/golden/make_golden.py) pins the bytes.
"""
from __future__ import annotations

import json
import os
import subprocess
import time
from collections import defaultdict
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "bin")

DEFAULT_CONFIG = {"hscale": 1.0, "fscale": 0.0, "time": 0, "itrs": -1, "k_moves": -1,
                  "threads": 0, "verbose": False, "debug": False, "thread_alloc": False,
                  "no_cache": False}                     # process_query.py:149-160

HEADER = ["expe", "n_expanded", "n_inserted", "n_touched", "n_updated", "n_surplus", "plen",
          "finished", "t_receive", "t_astar", "t_search", "t_prepare", "t_partition",
          "size"]                                        # process_query.py:197-212


def read_p2p(path):
    """process_query.read_p2p (:22-32)."""
    reqs = []
    with open(path) as f:
        for line in f:
            if not line.strip() or line[0] != "q":
                continue
            reqs.append([int(x) for x in line.split()[1:]])
    return reqs


def get_node_num(xyfile):
    """process_query.get_node_num (:126-130)."""
    with open(xyfile) as f:
        line = f.readlines()[3]
        _, num, _, _ = line.split(" ")
    return int(num)


def gen_distribute_conf(nodenum, maxworker, partmethod, partkey):
    """Run our bin/gen_distribute_conf exactly as make_parts does (:46-47)."""
    cmd = [os.path.join(BIN, "gen_distribute_conf"), "--nodenum", str(nodenum), "--maxworker",
           str(maxworker), "--partmethod", partmethod, "--partkey", str(partkey)]
    p = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    out = p.stdout
    if out.endswith("\n"):          # subprocess.getstatusoutput strips one newline
        out = out[:-1]
    return p.returncode, out


def make_parts(reqs, nodenum, maxworker, partmethod, partkey, activew=-1):
    """process_query.make_parts (:35-63), including its empty-worker compaction."""
    code, out = gen_distribute_conf(nodenum, maxworker, partmethod, partkey)
    if code:
        return code, out
    node2worker = {}
    for line in out.split("\n")[1:]:
        node, wid, bid, bidx = map(int, line.split(","))
        node2worker[node] = wid
    groups = defaultdict(list)
    for s, t in reqs:
        wid = node2worker[t]
        if activew == -1 or wid == activew:
            groups[wid].append([s, t])
    parts = [groups[i] for i in range(maxworker) if groups.get(i) is not None]
    return code, parts


def query_file_bytes(reqs):
    """send_queries (:93-96)."""
    return f"{len(reqs)}\n" + "".join("{} {}\n".format(*x) for x in reqs)


def remote_script(config_text, answer, fifo):
    """send_remote (:66-79): the bash script piped to the worker."""
    return (f"mkfifo {answer}\n" + f"cat <<CONF > {fifo}\n" + config_text + "CONF\n" +
            f"cat {answer}\n" + f"rm {answer}")


def send_queries(hostname, workerid, nfs, config, dname, reqs, script_dir):
    """send_queries (:82-111) with `ssh host 'bash -s'` replaced by local bash."""
    fname = os.path.join(script_dir, f"query.{hostname}{workerid}")
    qname = os.path.join(nfs, f"query.{hostname}{workerid}")
    fifo = f"/tmp/worker{workerid}.fifo"
    answer = f"/tmp/worker{workerid}.answer"
    conf = json.dumps(config) + "\n" + "{} {} {}\n".format(qname, answer, dname)
    t0 = time.perf_counter()
    with open(qname, "w") as f:
        f.write(query_file_bytes(reqs))
    t_prepare = time.perf_counter() - t0
    with open(fname, "w") as f:
        f.write(remote_script(conf, answer, fifo))
    t0 = time.perf_counter()
    p = subprocess.run(f"bash -s < {fname}", shell=True, stdout=subprocess.PIPE,
                       stderr=subprocess.STDOUT, text=True, timeout=300)
    t_partition = time.perf_counter() - t0
    out = p.stdout[:-1] if p.stdout.endswith("\n") else p.stdout
    res = out.split(",") if p.returncode == 0 else ""
    if p.returncode == 0:
        os.remove(qname)
    os.remove(fname)
    return (*res, t_prepare * 1e9, t_partition * 1e9, len(reqs))


def run(conf, config=None, script_dir=None):
    """process_query.run (:132-194) for local workers.  The reference writes
    each worker's bash script to the head node's cwd under the query file's
    basename (process_query.py:83-84,70), so script_dir must not be the NFS
    directory."""
    import tempfile
    script_dir = script_dir or tempfile.mkdtemp(prefix="head-")
    assert os.path.realpath(script_dir) != os.path.realpath(conf["nfs"])
    config = dict(DEFAULT_CONFIG if config is None else config)
    hosts = conf["workers"]
    maxworker = len(hosts)
    nodenum = get_node_num(conf["xy_file"])
    reqs = read_p2p(conf["scenfile"])
    code, parts = make_parts(reqs, nodenum, maxworker, conf["partmethod"], conf["partkey"])
    assert code == 0, parts
    stats = []
    for dname in conf["diffs"]:
        with ThreadPoolExecutor(maxworker) as pool:
            futs = [pool.submit(send_queries, h, w, conf["nfs"], config, dname, part,
                                script_dir)
                    for h, w, part in zip(hosts, range(maxworker), parts) if len(part) > 0]
            stats.append([f.result() for f in futs])
    return parts, stats


def wait_ready(proc, timeout=60):
    """Block until a resident fifo_auto prints its "listening" line; returns
    its stdout so far.  Reads the raw pipe (os.read after select): a buffered
    readline can swallow several lines at once, after which select never
    reports the ones left in Python's buffer."""
    import select
    fd = proc.stdout.fileno()
    t0 = time.time()
    buf = b""
    while time.time() - t0 < timeout:
        r, _, _ = select.select([fd], [], [], 1.0)
        if r:
            chunk = os.read(fd, 65536)
            if not chunk:
                break
            buf += chunk
            if b"listening" in buf:
                return buf.decode(errors="replace")
        if proc.poll() is not None:
            break
    proc.kill()
    err = proc.stderr.read() if proc.stderr else ""
    raise AssertionError(f"fifo_auto did not come up: {buf.decode(errors='replace')} {err}")
