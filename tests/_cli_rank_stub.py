"""A rank process for tests/test_cli_launcher.py: what `python -m vaeb_amd <argv>` runs in
each child of cli.main's launcher (dp.spawn_ranks), with the HIP library replaced by the
recording stand-in of tests/test_cli_dp.py (gloo all-reduce, no GPU).  Writes what it saw
(its rank environment, its stdout) to $STUB_OUT/rank<r>.json.  STUB_MODE=fail makes rank 1
exit 3 before joining the group; STUB_MODE=hang makes rank 1 exit 0 at once while rank 0
never returns; STUB_MODE=slowlead makes rank 0's .mdl save sleep STUB_SLOW_S seconds first."""
import io
import json
import os
import sys
import time
from contextlib import redirect_stdout

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)


def main():
    rank = int(os.environ["RANK"])
    mode = os.environ.get("STUB_MODE", "")
    env = {k: os.environ.get(k) for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    out_dir = os.environ["STUB_OUT"]
    with open(os.path.join(out_dir, f"started{rank}"), "w") as f:
        f.write(str(os.getpid()))
    if mode == "fail" and rank == 1:
        sys.exit(3)
    if mode == "hang":
        if rank == 1:
            sys.exit(0)
        time.sleep(600)
    from test_cli_dp import RecordingCtx
    from vaeb_amd import _lib, cli
    _lib.Context = RecordingCtx
    if mode == "slowlead" and rank == 0:
        # rank 0's lead-only tail (the .mdl write) outlasts the straggler deadline
        from vaeb_amd import model as M
        save = M.VAEB.save

        def slow_save(self, f):
            time.sleep(float(os.environ.get("STUB_SLOW_S", "4")))
            save(self, f)
        M.VAEB.save = slow_save
    buf = io.StringIO()
    with redirect_stdout(buf):
        cli.main(sys.argv[1:])
    m = RecordingCtx.made[-1]
    with open(os.path.join(out_dir, f"rank{rank}.json"), "w") as f:
        json.dump({"env": env, "stdout": buf.getvalue(), "cfg": m.cfg,
                   "theta": m.get_params().astype(float).tolist()[:64]}, f)


if __name__ == "__main__":
    main()
