"""Launcher: ``python -m cs230_distributed_machine_learning_amd.serve --gpus 8 --port 5001``.

One process per GPU (torch.distributed over RCCL).  Rank 0 runs the controller, the
HTTP gateway (same routes as the reference master + scheduler) and is itself a worker;
ranks 1..N-1 are workers.  With ``--gpus 1`` (or no GPU) everything runs in one
process with the local runner.  Replaces the reference's docker-compose topology of
master + scheduler + 4 workers + Kafka + Redis (aws-prod/docker-compose.yml).
"""
from __future__ import annotations

import argparse
import os
import subprocess
import sys


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="distributed-ml (MI355X) service")
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--master-port", type=int, default=29541)
    from .config import Config

    Config.add_cli(ap)
    args = ap.parse_args(argv)
    if args.gpus > 1 and int(os.environ.get("WORLD_SIZE", "1")) == 1:
        # re-launch one rank per GPU before touching the GPU in this process
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
               "--master-addr", "127.0.0.1", "--master-port", str(args.master_port), "-m",
               "cs230_distributed_machine_learning_amd.serve"] + (argv if argv is not None else sys.argv[1:])
        env = dict(os.environ)
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        return subprocess.call(cmd, env=env)

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
    else:
        worker_loop(core)
    dist.destroy()
    return 0


if __name__ == "__main__":
    sys.exit(main())
