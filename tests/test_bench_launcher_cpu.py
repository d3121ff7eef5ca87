"""bench.py's self-launcher (`python bench.py --gpus N` without torchrun):
argument handling, environment, output relay and exit codes, on the CPU with
stand-in rank programs (no GPU is touched)."""
from __future__ import annotations

import json
import os
import subprocess
import sys
import time

import bench

RANK_ENV = ("import os, json, sys; e = {k: os.environ.get(k) for k in "
            "('RANK', 'LOCAL_RANK', 'WORLD_SIZE', 'MASTER_ADDR', 'MASTER_PORT', 'ZK_BENCH_LAUNCHER')}; ")


def test_all_ranks_ok_relays_rank0_line():
    code = RANK_ENV + "print('banner on rank', e['RANK'], file=sys.stderr); " \
                      "print(json.dumps(e)) if e['RANK'] == '0' else None"
    rc, text = bench.spawn_ranks(4, [sys.executable, "-c", code])
    assert rc == 0
    lines = text.splitlines()
    assert len(lines) == 1  # only rank 0's stdout is captured
    e = json.loads(lines[0])
    assert e["RANK"] == "0" and e["LOCAL_RANK"] == "0" and e["WORLD_SIZE"] == "4"
    assert e["MASTER_ADDR"] == "127.0.0.1" and int(e["MASTER_PORT"]) > 0
    assert e["ZK_BENCH_LAUNCHER"] == "self"


def test_every_rank_sees_its_own_rank(tmp_path):
    code = RANK_ENV + f"open(os.path.join({str(tmp_path)!r}, e['RANK']), 'w').write(json.dumps(e))"
    rc, _ = bench.spawn_ranks(8, [sys.executable, "-c", code])
    assert rc == 0
    seen = [json.load(open(tmp_path / str(r))) for r in range(8)]
    assert [s["LOCAL_RANK"] for s in seen] == [str(r) for r in range(8)]
    assert len({s["MASTER_PORT"] for s in seen}) == 1  # one rendezvous


def test_failing_rank_ends_the_job_with_its_code():
    # rank 2 fails at once; the others would wait forever (as at a barrier)
    code = "import os, sys, time; r = int(os.environ['RANK']); sys.exit(7) if r == 2 else time.sleep(600)"
    t0 = time.monotonic()
    rc, text = bench.spawn_ranks(4, [sys.executable, "-c", code], grace_s=1.0)
    assert rc == 7
    assert time.monotonic() - t0 < 60
    assert text == ""


def test_signal_death_maps_to_128_plus_signal():
    code = "import os, signal; os.kill(os.getpid(), signal.SIGSEGV) if os.environ['RANK'] == '1' else None"
    rc, _ = bench.spawn_ranks(2, [sys.executable, "-c", code], grace_s=5.0)
    assert rc == 128 + 11


def test_rank0_failure_after_printing_is_a_failure():
    code = "import os, sys; print('{}'); sys.exit(3 if os.environ['RANK'] == '0' else 0)"
    rc, text = bench.spawn_ranks(2, [sys.executable, "-c", code], grace_s=5.0)
    assert rc == 3


def test_bench_main_self_launch_relays_failure_without_gpu():
    """`python bench.py --gpus 2` in this GPU-less container: the parent starts
    two rank processes (it never imports torch), both fail to create a device
    context, and the parent exits non-zero with nothing on stdout."""
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, bench.__file__, "--gpus", "2", "--steps", "1", "--warmup", "0"],
                       env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode != 0
    assert r.stdout == ""
    assert "bench launcher: rank" in r.stderr


def test_world_mismatch_is_refused():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, bench.__file__, "--gpus", "4"], env=env, capture_output=True, text=True,
                       timeout=120)
    assert r.returncode != 0
    assert "WORLD_SIZE=2" in r.stderr


def test_timeout_kills_hung_ranks():
    """The N>1 bench's peer-reduction side leg starts its ranks with a time
    limit: ranks still running after it are killed and the leg reads as failed
    (124), so a hang there cannot hold the headline line."""
    code = "import time; time.sleep(600)"
    t0 = time.monotonic()
    rc, text = bench.spawn_ranks(2, [sys.executable, "-c", code], grace_s=1.0, timeout_s=2.0)
    assert rc == 124
    assert time.monotonic() - t0 < 60
    assert text == ""


def test_timeout_does_not_touch_ranks_that_finish():
    code = "import os; print('{\"ok\": 1}') if os.environ['RANK'] == '0' else None"
    rc, text = bench.spawn_ranks(2, [sys.executable, "-c", code], timeout_s=120.0)
    assert rc == 0 and json.loads(text.splitlines()[-1]) == {"ok": 1}


def test_elastic_agent_settings_are_not_inherited(monkeypatch):
    """Rank 0 of a torch.distributed.run job starts the peer-reduction side leg
    through spawn_ranks: its children must host their own rendezvous store,
    so the elastic agent's variables (TORCHELASTIC_USE_AGENT_STORE above all)
    are not passed down."""
    monkeypatch.setenv("TORCHELASTIC_USE_AGENT_STORE", "True")
    monkeypatch.setenv("TORCHELASTIC_RUN_ID", "none")
    monkeypatch.setenv("GROUP_WORLD_SIZE", "1")
    monkeypatch.setenv("ROLE_RANK", "3")
    code = ("import os, json; print(json.dumps(sorted(k for k in os.environ if k.startswith("
            "('TORCHELASTIC_', 'GROUP_WORLD', 'ROLE_')))))")
    rc, text = bench.spawn_ranks(2, [sys.executable, "-c", code])
    assert rc == 0
    assert json.loads(text.splitlines()[-1]) == []
