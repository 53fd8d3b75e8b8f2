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
    seeds = [bench.frame_id(rank, f, 4) for f in range(4)]
    # the verification of a row-sharded output: each rank checks its own row
    # bands against the fixture's 8 band hashes; a bad rank fails every rank
    import numpy as np, torch
    from __graft_entry__ import load_package
    pkg = load_package()
    w, h = 64, 16
    full = pkg.synth_frame(w * h, 5)
    fix = {"ct": [1, 2], "out_fnv": "%%016x" %% pkg.fnv1a64(full),
           "band_fnv": ["%%016x" %% pkg.fnv1a64(full[b * 2 * w:(b + 1) * 2 * w]) for b in range(8)]}
    r0, r1 = bench.row_range(h, rank, world)
    mine = torch.from_numpy(full[r0 * w:r1 * w].view(np.int32).copy())
    good = bench.check_frame(pkg, mine, [1, 2], fix, rows=(r0, r1), h=h, world=world, rank=rank)
    bad_ct = bench.check_frame(pkg, mine, [1, 3], fix, rows=(r0, r1), h=h, world=world, rank=rank)
    if rank == 1:
        mine[7] ^= 1
    tampered = bench.check_frame(pkg, mine, [1, 2], fix, rows=(r0, r1), h=h, world=world, rank=rank)
    agree = bench.all_ranks_ok(tampered, world, "cpu")
    print(json.dumps({"rank": rank, "dt": dt, "dtmax": dtmax, "seeds": seeds, "good": good,
                      "bad_ct": bad_ct, "tampered": tampered, "agree": agree}), flush=True)
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
    # row-band verification: each rank's own bands; one bad rank fails both
    assert all(o["good"] is True and o["bad_ct"] is False for o in outs)
    assert outs[0]["tampered"] is True and outs[1]["tampered"] is False
    assert outs[0]["agree"] is False and outs[1]["agree"] is False


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


def test_bench_gpus_2_launches_two_ranks():
    """`bench.py --gpus 2` with no torchrun environment starts two ranks by
    itself (torch.distributed.run; gloo on CPU, RCCL on the GPU box), every
    rank checks the world size, and rank 0 prints ONE line with n_gpus 2."""
    import json
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK",
                                                             "MASTER_ADDR", "MASTER_PORT")}
    env["CUDA_VISIBLE_DEVICES"] = ""
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3",
                        "--dry-run"], env=env, capture_output=True, text=True, timeout=180)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["dry_run"] is True
    # the slower rank (20 ms per step) bounds the reported time
    assert d["ms_per_step"] >= 20.0


def test_bench_world_size_must_match_gpus():
    """A torchrun environment whose world size differs from --gpus is refused
    (the driver's --gpus N line can only come from N ranks)."""
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0", CUDA_VISIBLE_DEVICES="")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run"],
                       env=env, capture_output=True, text=True, timeout=120)
    assert p.returncode != 0 and "--gpus 2" in p.stderr
