"""The CLI's own rank launcher end to end, on CPU.

`python -m vaeb_amd ... --world_size 2` with no WORLD_SIZE in the environment goes through
cli.main -> dp.spawn_ranks(2, dp.module_cmd(argv)) (cli.py main; the reference's device
selection is run_on_gpu.sh:2 around VAEB.py:601-608).  Here module_cmd is replaced by a stub
rank script (tests/_cli_rank_stub.py) that runs cli.main in each child with the recording
stand-in for the HIP library, so the launcher itself -- environment, rendezvous, exit codes,
stopping the other ranks -- is what runs.  Checked:
* two children with RANK / LOCAL_RANK 0 and 1, WORLD_SIZE 2, one rendezvous on 127.0.0.1;
* rank 0 alone prints; both ranks end with the same parameters;
* a failing rank makes main exit with its code, and the other rank (blocked in the group
  rendezvous) is killed rather than left hanging;
* a rank still running after its peer exited 0 is stopped after the straggler deadline
   with dp.RANK_HUNG;
* rank 0's lead-only tail (the .mdl save) longer than that deadline is not a hang: the ranks
  leave train_model together through a final barrier.
"""
import os
import sys
import time

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
STUB = os.path.join(HERE, "_cli_rank_stub.py")
ARGV = ['--n_epochs', '1', '--synthetic', '--continuous', '--n_latent', '2', '--world_size', '2']


@pytest.fixture
def launcher(monkeypatch, tmp_path):
    from vaeb_amd import dp
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "STUB_MODE"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("STUB_OUT", str(tmp_path))
    monkeypatch.setattr(dp, "module_cmd", lambda argv: [sys.executable, STUB] + list(argv))
    monkeypatch.chdir(tmp_path)
    return tmp_path


def _alive(pid):
    try:
        os.kill(pid, 0)
    except ProcessLookupError:
        return False
    try:   # a zombie is not running either
        with open(f"/proc/{pid}/stat") as f:
            return f.read().split()[2] != "Z"
    except FileNotFoundError:
        return False


def test_cli_launcher_spawns_two_ranks(launcher):
    import json
    from vaeb_amd import cli
    assert cli.main(list(ARGV)) == (None, None)       # the parent made no model
    r = [json.load(open(launcher / f"rank{k}.json")) for k in (0, 1)]
    for k in (0, 1):
        e = r[k]["env"]
        assert (e["RANK"], e["LOCAL_RANK"], e["WORLD_SIZE"]) == (str(k), str(k), "2")
        assert e["MASTER_ADDR"] == "127.0.0.1"
    assert r[0]["env"]["MASTER_PORT"] == r[1]["env"]["MASTER_PORT"]
    # strong scaling (the CLI's default): the 100-row minibatch as 50 + 50
    assert (r[0]["cfg"]["B"], r[0]["cfg"]["row_offset"]) == (50, 0)
    assert (r[1]["cfg"]["B"], r[1]["cfg"]["row_offset"]) == (50, 50)
    assert "Epoch 0 :" in r[0]["stdout"] and r[1]["stdout"] == ""
    assert r[0]["theta"] == r[1]["theta"]


def test_cli_launcher_failing_rank_stops_the_other(launcher, monkeypatch):
    from vaeb_amd import cli
    monkeypatch.setenv("STUB_MODE", "fail")
    t0 = time.monotonic()
    with pytest.raises(SystemExit) as ei:
        cli.main(list(ARGV))
    assert ei.value.code == 3
    assert time.monotonic() - t0 < 60
    if os.path.exists(launcher / "started0"):          # (it may be killed before it got that far)
        assert not _alive(int(open(launcher / "started0").read()))   # killed, not left in the rendezvous
    assert not os.path.exists(launcher / "rank0.json")


def test_cli_launcher_straggler_deadline(launcher, monkeypatch):
    from vaeb_amd import cli, dp
    monkeypatch.setenv("STUB_MODE", "hang")
    monkeypatch.setenv("VAEB_RANK_DEADLINE_S", "2")
    t0 = time.monotonic()
    with pytest.raises(SystemExit) as ei:
        cli.main(list(ARGV))
    assert ei.value.code == dp.RANK_HUNG
    assert time.monotonic() - t0 < 30
    assert not _alive(int(open(launcher / "started0").read()))


def test_cli_launcher_slow_lead_tail_is_not_a_straggler(launcher, monkeypatch):
    from vaeb_amd import cli
    monkeypatch.setenv("STUB_MODE", "slowlead")
    monkeypatch.setenv("STUB_SLOW_S", "4")
    monkeypatch.setenv("VAEB_RANK_DEADLINE_S", "2")
    assert cli.main(list(ARGV) + ['--save_file', 'm.mdl']) == (None, None)
    assert os.path.exists(launcher / "rank0.json") and os.path.exists(launcher / "rank1.json")
    assert os.path.getsize(launcher / "m.mdl") > 0
