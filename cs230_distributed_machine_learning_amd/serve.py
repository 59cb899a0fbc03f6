"""Launcher: ``python -m cs230_distributed_machine_learning_amd.serve --gpus 8 --port 5001``.

One process per GPU (torch.distributed over RCCL).  Rank 0 runs the controller, the
HTTP gateway (same routes as the reference master + scheduler), the dispatcher, and is
itself a worker; ranks 1..N-1 are workers.  With ``--gpus 1`` (or no GPU) everything
runs in one process with the local runner.  Replaces the reference's docker-compose
topology of master + scheduler + 4 workers + Kafka + Redis (aws-prod/docker-compose.yml).

The parent process (which never touches a GPU) starts the ranks as its own children
and supervises them: when a worker rank dies, the dispatcher on rank 0 re-queues its work
to the survivors and re-forms the process group without it, and the supervisor starts a
FRESH child on the same GPU that joins the running service (``--join``; never an exec of
the dead process), with bounded restarts per GPU (``--respawn``, default 3) and a
back-off; rank 0 then takes the replacement into the next communicator generation, so
the GPU gets the same service as every other (reference: a restarted worker re-registers
and is served like any other, aws-prod/worker/worker.py:90-112 -> scheduler.py:105-117).
Only rank 0 exiting ends the service.  (torchrun's elastic agent would instead tear the
whole group down, controller included, when any worker exits.)

Extra capacity can join a running service at any time (elastic membership, reference
aws-prod/scheduler/scheduler.py:105-117):
``python -m cs230_distributed_machine_learning_amd.serve --join 127.0.0.1:29541 --device cuda:3``
"""
from __future__ import annotations

import argparse
import os
import signal
import subprocess
import sys
import time


def _supervise(args, argv) -> int:
    """Start one child per rank (before any GPU call here) and supervise them."""
    env0 = dict(os.environ)
    env0.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env0.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(args.master_port), WORLD_SIZE=str(args.gpus))
    procs = []
    for r in range(args.gpus):
        env = dict(env0, RANK=str(r), LOCAL_RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, "-m", "cs230_distributed_machine_learning_amd.serve"] + argv,
                                      env=env))

    def stop(*_):
        for p in procs:
            if p.poll() is None:
                p.terminate()

    signal.signal(signal.SIGTERM, stop)
    slot = {r: procs[r] for r in range(1, args.gpus)}   # GPU r -> its current worker process
    restarts = {r: 0 for r in slot}
    due = {}                                             # GPU r -> time its replacement starts
    dev_kind = "cpu" if (getattr(args, "device", None) == "cpu") else "cuda"
    try:
        while True:
            rc0 = procs[0].poll()
            if rc0 is not None:          # the service (rank 0) ended: stop the workers
                stop()
                deadline = time.time() + 30
                for p in procs[1:]:
                    try:
                        p.wait(timeout=max(0.1, deadline - time.time()))
                    except subprocess.TimeoutExpired:
                        p.kill()
                return rc0
            now = time.time()
            for r, p in list(slot.items()):
                if p is None or p.poll() is None:
                    continue
                rc = p.returncode
                slot[r] = None
                if rc == 0:              # a graceful leave (/unsubscribe): not restarted
                    print(f"[serve] worker on GPU {r} left", file=sys.stderr, flush=True)
                    continue
                if restarts[r] >= args.respawn:
                    print(f"[serve] worker on GPU {r} exited with code {rc}; restart budget spent, GPU left idle",
                          file=sys.stderr, flush=True)
                    continue
                restarts[r] += 1
                due[r] = now + min(30.0, args.respawn_backoff * 2 ** (restarts[r] - 1))
                print(f"[serve] worker on GPU {r} exited with code {rc}; rank 0 re-queues its work, a replacement "
                      f"joins in {due[r] - now:.1f}s (restart {restarts[r]}/{args.respawn})", file=sys.stderr,
                      flush=True)
            for r, t in list(due.items()):
                if now < t:
                    continue
                del due[r]
                env = dict(env0, WORLD_SIZE="1", RANK="0", LOCAL_RANK=str(r))
                dev = "cpu" if dev_kind == "cpu" else f"cuda:{r}"
                cmd = [sys.executable, "-m", "cs230_distributed_machine_learning_amd.serve",
                       "--join", f"127.0.0.1:{args.master_port}", "--device", dev]
                p = subprocess.Popen(cmd, env=env)
                procs.append(p)
                slot[r] = p
            time.sleep(0.5)
    except KeyboardInterrupt:
        stop()
        return 130


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="distributed-ml (MI355X) service")
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--master-port", type=int, default=29541)
    ap.add_argument("--join", default=None, metavar="HOST:PORT",
                    help="join a running service (its --master-port) as an extra worker")
    ap.add_argument("--respawn", type=int, default=3,
                    help="restarts per GPU of a worker rank that died (a fresh process that joins)")
    ap.add_argument("--respawn-backoff", type=float, default=1.0,
                    help="seconds before the first restart of a GPU's worker (doubles per restart)")
    from .config import Config

    Config.add_cli(ap)
    argv = list(argv if argv is not None else sys.argv[1:])
    args = ap.parse_args(argv)
    if args.join:
        from .parallel.runner import join_cluster
        import torch

        host, _, port = args.join.rpartition(":")
        dev = torch.device(args.device if args.device not in (None, "auto") else
                           ("cuda:0" if torch.cuda.is_available() else "cpu"))
        if dev.type == "cuda":
            torch.cuda.set_device(dev)
        wid = join_cluster(host or "127.0.0.1", int(port), dev)
        print(f"[serve] worker {wid} left the cluster", file=sys.stderr)
        return 0
    if args.gpus > 1 and int(os.environ.get("WORLD_SIZE", "1")) == 1:
        return _supervise(args, argv)

    cfg = Config.from_args(args)
    from .utils.log import get_logger

    log = get_logger("dml.serve", cfg.log_dir)
    if int(os.environ.get("WORLD_SIZE", "1")) == 1:
        from .engine.service import Controller
        from .gateway.app import serve

        ctl = Controller(cfg)
        log.info("serving on http://%s:%d (device %s)", cfg.host, cfg.port, cfg.resolved_device())
        serve(ctl, cfg.host, cfg.port, block=True)
        return 0

    from .parallel import dist
    from .parallel.runner import DistributedRunner, WorkerCore, worker_loop

    inf = dist.init(want_gpu=cfg.device != "cpu")
    core = WorkerCore(inf.device)
    if inf.rank == 0:
        from .engine.service import Controller
        from .gateway.app import serve

        runner = DistributedRunner(core)
        ctl = Controller(cfg, runner=runner)
        serve(ctl, cfg.host, cfg.port, block=False)
        log.info("rank 0: serving on http://%s:%d with %d ranks", cfg.host, cfg.port, inf.world)
        try:
            runner.serve_forever()
        except KeyboardInterrupt:
            runner.shutdown()
        if runner.dead or runner.group_broken or runner.gen > 0:
            os._exit(0)   # a peer is gone or the group was re-formed: a teardown could wait for it
    else:
        worker_loop(core)
    dist.destroy()
    return 0


if __name__ == "__main__":
    sys.exit(main())
