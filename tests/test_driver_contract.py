"""Drop-in boundary on CPU: our executables' I/O against fixtures captured from
the reference's own Python drivers (tests/golden/make_golden.py)."""
import hashlib
import json
import os
import subprocess

import pytest

import driver_harness as H

FX = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "driver_fixtures.json")))


@pytest.mark.parametrize("case", FX["make_parts"], ids=lambda c: "{nodenum}-{maxworker}-{partmethod}{partkey}".format(**c))
def test_make_parts_matches_reference(case):
    code, parts = H.make_parts(case["reqs"], case["nodenum"], case["maxworker"],
                               case["partmethod"], case["partkey"], case.get("activew", -1))
    assert code == 0
    assert parts == case["parts"]


@pytest.mark.parametrize("case", [c for c in FX["make_parts"] if "node2worker" in c],
                         ids=lambda c: "{nodenum}-{maxworker}-{partmethod}{partkey}".format(**c))
def test_gen_distribute_conf_format(case):
    p = subprocess.run([os.path.join(H.BIN, "gen_distribute_conf"), "--nodenum", str(case["nodenum"]),
                        "--maxworker", str(case["maxworker"]), "--partmethod", case["partmethod"],
                        "--partkey", str(case["partkey"])], capture_output=True, text=True)
    assert p.returncode == 0 and p.stderr == ""          # getstatusoutput merges stderr
    lines = p.stdout.rstrip("\n").split("\n")
    assert lines[0] == "node,wid,bid,bidx" and len(lines) == case["nodenum"] + 1
    got = {}
    for line in lines[1:]:
        node, wid, bid, bidx = map(int, line.split(","))
        got[str(node)] = wid
    assert got == case["node2worker"]


def test_partition_alias_and_errors():
    p = subprocess.run([os.path.join(H.BIN, "gen_distribute_conf"), "--nodenum", "5",
                        "--maxworker", "2", "--partition", "div", "--partkey", "2"],
                       capture_output=True, text=True)
    assert p.returncode == 0 and p.stdout.count("\n") == 6
    p = subprocess.run([os.path.join(H.BIN, "gen_distribute_conf"), "--nodenum", "5"],
                       capture_output=True, text=True)
    assert p.returncode != 0


def test_query_file_and_script_bytes():
    sq = FX["send_queries"]
    assert H.query_file_bytes(sq["reqs"]) == sq["query_file"]
    # fixture dicts are stored key-sorted; the wire order is process_query.py:149-160's
    conf = json.dumps(H.DEFAULT_CONFIG) + "\n" + "{} {} {}\n".format(
        "<NFS>/query.localhost1", "/tmp/worker1.answer", sq["dname"])
    assert H.remote_script(conf, "/tmp/worker1.answer", "/tmp/worker1.fifo") == sq["script"]
    assert sq["config"] == H.DEFAULT_CONFIG
    assert sq["result_len"] == 13 and len(FX["answer_line"].split(",")) == 10


def test_generated_files_parse_like_reference(tmp_path):
    f = FX["files"]
    prefix = str(tmp_path / "g")
    subprocess.run([os.path.join(H.BIN, "gen_synth"), *f["gen_synth_args"][:6], "--out", prefix,
                    *f["gen_synth_args"][6:]], check=True, capture_output=True)
    assert hashlib.sha256(open(prefix + ".xy", "rb").read()).hexdigest() == f["xy_sha256"]
    assert hashlib.sha256(open(prefix + ".scen", "rb").read()).hexdigest() == f["scen_sha256"]
    assert H.get_node_num(prefix + ".xy") == f["get_node_num"]
    assert H.read_p2p(prefix + ".scen") == f["read_p2p"]
