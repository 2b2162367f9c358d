"""Generate driver-contract golden fixtures by running the REFERENCE Python.

Run in the build container only (it reads /root/reference; the GPU box never
does):  python tests/golden/make_golden.py

It imports the reference's own process_query.py (which imports args.py and
timer.py) and feeds it inputs produced by OUR tools, so the fixtures pin how
the unmodified reference driver consumes our gen_distribute_conf output, our
.xy header and our .scen files, and exactly which bytes it sends to a worker:
  - make_parts (process_query.py:35-63) routing, incl. the empty-worker case
  - send_queries/send_remote (process_query.py:66-111): the query file bytes,
    the bash script bytes, the ssh command, the result tuple layout
  - get_node_num (process_query.py:126-130) and read_p2p (:22-32)
ssh is never run: process_query.getstatusoutput is wrapped so that `ssh ...`
commands are captured and answered with a fixed stats line, while the
`./bin/gen_distribute_conf` call runs our real binary.
"""
import hashlib
import json
import os
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"


def main():
    subprocess.run(["make", "-C", ROOT, "bins"], check=True, stdout=subprocess.DEVNULL)
    sys.argv = ["process_query.py"]          # args.py parses argv at import
    sys.path.insert(0, REF)
    os.chdir(ROOT)                           # make_parts runs ./bin/gen_distribute_conf
    import process_query as pq               # noqa: E402  (reference module)

    real = pq.getstatusoutput
    captured = []
    ANSWER = "11,0,0,0,0,11,2,1234,0,5678"

    def fake(cmd):
        if cmd.startswith("ssh "):
            script = cmd.split("< ", 1)[1]
            with open(script) as f:
                captured.append({"cmd": cmd, "script": f.read()})
            return 0, ANSWER
        return real(cmd)

    pq.getstatusoutput = fake
    fx = {"answer_line": ANSWER}

    # make_parts over several partitions (node2worker is a module global)
    reqs = [[0, 5], [1, 6], [2, 7], [3, 8], [4, 9], [9, 0], [7, 7], [6, 2]]
    cases = []
    for nodenum, W, method, key in [(10, 3, "mod", 3), (10, 3, "div", 3), (10, 2, "mod", 9),
                                    (10, 2, "div", 4), (25, 4, "mod", 100), (10, 1, "div", 1)]:
        pq.node2worker.clear()
        code, parts = pq.make_parts(reqs, nodenum, W, method, key, -1)
        assert code == 0, parts
        cases.append({"nodenum": nodenum, "maxworker": W, "partmethod": method, "partkey": key,
                      "reqs": reqs, "parts": parts,
                      "node2worker": {str(k): v for k, v in sorted(pq.node2worker.items())}})
    # empty-worker case: W=3, mod 3, no target owned by worker 0
    pq.node2worker.clear()
    code, parts = pq.make_parts([[0, 4], [2, 5]], 6, 3, "mod", 3, -1)
    cases.append({"nodenum": 6, "maxworker": 3, "partmethod": "mod", "partkey": 3,
                  "reqs": [[0, 4], [2, 5]], "parts": parts, "empty_worker": True})
    # activew filter
    pq.node2worker.clear()
    code, parts = pq.make_parts(reqs, 10, 3, "mod", 3, 1)
    cases.append({"nodenum": 10, "maxworker": 3, "partmethod": "mod", "partkey": 3,
                  "reqs": reqs, "parts": parts, "activew": 1})
    fx["make_parts"] = cases

    # send_queries: query file + script bytes
    with tempfile.TemporaryDirectory() as nfs:
        conf = {"hscale": 1.0, "fscale": 0.0, "time": 0, "itrs": -1, "k_moves": -1,
                "threads": 0, "verbose": False, "debug": False, "thread_alloc": False,
                "no_cache": False}
        qpath = os.path.join(nfs, "query.localhost1")
        seen = {}
        real_open = open

        def spy_open(path, mode="r", *a, **k):
            fh = real_open(path, mode, *a, **k)
            if path == qpath and "w" in mode:
                seen["q"] = fh
            return fh

        import builtins
        builtins.open = spy_open
        try:
            old = os.remove
            removed = []
            os.remove = lambda p: (removed.append(p), old(p))[1] if p != qpath else (
                seen.__setitem__("qbytes", real_open(p).read()), removed.append(p), old(p))
            res = pq.send_queries("localhost", 1, nfs, conf, "./data/x.xy.diff", [[2, 7], [5, 8]])
        finally:
            builtins.open = real_open
            os.remove = old
        fx["send_queries"] = {
            "hostname": "localhost", "workerid": 1, "nfs": "<NFS>", "config": conf,
            "dname": "./data/x.xy.diff", "reqs": [[2, 7], [5, 8]],
            "query_file": seen["qbytes"],
            "script": captured[-1]["script"].replace(nfs, "<NFS>"),
            "cmd": captured[-1]["cmd"].replace(nfs, "<NFS>"),
            "result_len": len(res), "result_head": list(res[:10]), "result_size": res[-1],
        }
        if os.path.exists("query.localhost1"):
            os.remove("query.localhost1")       # send_remote leaves the script in cwd

    # get_node_num / read_p2p on our generated files
    with tempfile.TemporaryDirectory() as d:
        prefix = os.path.join(d, "g")
        subprocess.run([os.path.join(ROOT, "bin", "gen_synth"), "--width", "12", "--height", "9",
                        "--seed", "1", "--out", prefix, "--queries", "40"], check=True,
                       stdout=subprocess.DEVNULL)
        with open(prefix + ".xy", "rb") as f:
            xy_sha = hashlib.sha256(f.read()).hexdigest()
        with open(prefix + ".scen", "rb") as f:
            scen_sha = hashlib.sha256(f.read()).hexdigest()
        fx["files"] = {"gen_synth_args": ["--width", "12", "--height", "9", "--seed", "1",
                                          "--queries", "40"],
                       "xy_sha256": xy_sha, "scen_sha256": scen_sha,
                       "get_node_num": pq.get_node_num(prefix + ".xy"),
                       "read_p2p": pq.read_p2p(prefix + ".scen")}

    out = os.path.join(HERE, "driver_fixtures.json")
    with open(out, "w") as f:
        json.dump(fx, f, indent=1, sort_keys=True)
    print("wrote", out)


if __name__ == "__main__":
    main()
