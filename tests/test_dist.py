"""CPU, world_size 2 over gloo: the multi-rank harness of bench.py (one process
per GPU in production).  Each rank owns its own frames; the timed region is
bracketed by barriers; the reported time is the max over ranks; the value is
all ranks' pixels over that time ("scaling": "weak", no data-path collective)."""
import os
import socket
import subprocess
import sys
import textwrap

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

WORKER = textwrap.dedent("""
    import json, os, sys, time
    sys.path.insert(0, %(root)r)
    import bench
    rank, world, local = bench.init_dist()
    assert world == 2
    # ranks take different times; the harness must report the slower one
    delay = 0.05 * (rank + 1)
    dt = bench.timed_region(lambda: time.sleep(delay), 3, world, lambda: None)
    dtmax = bench.max_over_ranks(dt, world)
    seeds = [bench.frame_seed(rank, f) for f in range(4)]
    print(json.dumps({"rank": rank, "dt": dt, "dtmax": dtmax, "seeds": seeds}), flush=True)
    import torch.distributed as dist
    dist.destroy_process_group()
""")


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_rank_harness(tmp_path):
    import json
    script = tmp_path / "worker.py"
    script.write_text(WORKER % {"root": ROOT})
    port = free_port()
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE="2",
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), CUDA_VISIBLE_DEVICES="")
        procs.append(subprocess.Popen([sys.executable, str(script)], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = []
    for p in procs:
        o, e = p.communicate(timeout=120)
        assert p.returncode == 0, e
        outs.append(json.loads(o.strip().splitlines()[-1]))
    outs.sort(key=lambda d: d["rank"])
    # both ranks agree on the max, and it is the slow rank's time
    assert abs(outs[0]["dtmax"] - outs[1]["dtmax"]) < 1e-9
    assert outs[0]["dtmax"] >= 3 * 0.10
    assert outs[0]["dtmax"] >= max(o["dt"] for o in outs) - 1e-9
    # disjoint frames per rank
    assert not set(outs[0]["seeds"]) & set(outs[1]["seeds"])


def test_row_ranges_partition_the_frame():
    """Row-tile sharding (bench --mode rows): rank r owns rows [r*H/N, (r+1)*H/N)
    -- disjoint, ordered, covering every row, balanced to one row."""
    sys.path.insert(0, ROOT)
    import bench
    for h in (1, 7, 2160, 16384):
        for world in range(1, 9):
            rr = [bench.row_range(h, r, world) for r in range(world)]
            assert rr[0][0] == 0 and rr[-1][1] == h
            assert all(rr[i][1] == rr[i + 1][0] for i in range(world - 1))
            sizes = [b - a for a, b in rr]
            assert max(sizes) - min(sizes) <= 1
