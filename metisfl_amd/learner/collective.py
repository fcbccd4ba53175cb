"""One rank of an on-node collective federation, launched by
``DriverSession`` when the federation environment says ``DataPlane: rccl``
(one process per GPU, torch.distributed env from the driver).

Rank 0 fetches the driver's initial community model from the controller and
broadcasts it; every round the learners train their shards and average in
place with one RCCL all-reduce (parallel/federation.py), then evaluate the
new community model on their test shards; rank 0 reports each round (runtime
metadata, task lineages, the CommunityModelEvaluation) to the controller's
collective bookkeeping service, so the driver's ``monitor_federation`` /
``get_federation_statistics`` see the rounds.  The reference has no such data
plane: its learners always ship models through the controller
(driver_session.py:529-582 launches them with their GPUs).

Protocols: synchronous / semi-synchronous rounds (CollectiveFederation), or
the asynchronous protocol (AsyncCollectiveFederation.run_until: FedRec over
point-to-point transfers, one community version per completed task of any
learner; a rank's co-located learners are FedRec participants of their own).

Termination (the driver's TerminationSignals, driver_session.py:423-467):
FederationRounds (sync: rounds; async: community versions), the wall-clock
cutoff, the mean community-model test metric, or the driver's stop request;
rank 0 decides and the decision is broadcast, so every rank leaves after the
same round.

Failure handling: a ``FederatedModel`` checkpoint is written
every ``checkpoint_every`` rounds (staged on the device, written by a
background thread: parallel/checkpoint.py), a RankWatchdog exits the survivors of a
lost rank (exit code 75), and the driver relaunches them as FRESH processes
with ``resume_dir`` and the new world size.  ``fault`` ({"rank", "round"})
kills a rank at the start of a round (fault injection for tests).

    python -m metisfl_amd.learner.collective <job.json>
"""
from __future__ import annotations

import json
import os
import sys
import time

EXIT_INJECTED_FAULT = 17
# every rank exits with this after a blocking checkpoint when the driver asked
# for a new membership (a learner joins the running federation)
EXIT_REGROUP = 76


def _load_recipe(path):
    if not path:
        return None
    import cloudpickle  # the driver's own file (DriverSession._dump_recipe)
    with open(path, "rb") as f:
        return cloudpickle.load(f)


class _TorchNetDef:
    """A user TorchModelDef as a collective-plane model factory: each learner
    gets a TorchNet over its own module (models/torch_net.py)."""

    def __init__(self, model_def):
        self.model_def = model_def

    def get_model(self, batch_size: int, device="cpu", optimizer=None, seed: int = 0):
        from metisfl_amd.models.torch_net import TorchNet
        return TorchNet(self.model_def, batch_size, device=device, optimizer=optimizer, seed=seed)


def _load_model_def(job: dict):
    """The driver's model: a static-family JSON document, or (``model_kind``
    "torch") the user's cloudpickled TorchModelDef -- the driver's own file,
    as the reference's learners load the driver's pickled PyTorchDef
    (pytorch_model_ops.py:52-59)."""
    if job.get("model_kind", "static") == "torch":
        import cloudpickle
        with open(os.path.join(job["model_dir"], "model_def.pkl"), "rb") as f:
            return _TorchNetDef(cloudpickle.load(f))
    from metisfl_amd.models.model_def import StaticModelDef
    return StaticModelDef.load(job["model_dir"])


def _inject_fault(rank: int, at: int, fault: dict) -> None:
    """Fault injection (tests): leave now, with exit code EXIT_INJECTED_FAULT
    or -- ``"signal": "KILL"`` -- by SIGKILL, as the kernel's OOM killer
    would (exit -9)."""
    import signal
    how = str(fault.get("signal", "")).upper()
    print(f"[collective] fault injection: rank {rank} {'is SIGKILLed' if how == 'KILL' else 'exits'} at "
          f"{at}", flush=True)
    sys.stdout.flush()
    sys.stderr.flush()
    if how == "KILL":
        os.kill(os.getpid(), signal.SIGKILL)
    os._exit(EXIT_INJECTED_FAULT)


def _decision(comm, rank0_action: int) -> int:
    """Rank 0's decision after a round (0 continue, 1 stop, 2 regroup),
    identical on every rank."""
    import torch
    t = torch.tensor([float(rank0_action)], dtype=torch.float64, device=comm.device)
    comm.broadcast_(t, src=0)
    return int(round(t.item()))


def _he_decoder(fcfg, device):
    """The driver's CKKS key pair (rank 0 decrypts an encrypted initial
    model; on a GPU through the device kernels)."""
    if not (fcfg.secure_aggregation and fcfg.he_key_dir):
        return None
    from metisfl_amd.parallel.federation import setup_ckks
    scheme, _ = setup_ckks(None, fcfg)
    if device.type == "cuda":
        from metisfl_amd.encryption.device import AcceleratedCKKS
        return AcceleratedCKKS(scheme, device)
    return scheme


def _await_peer_verdict(wd) -> None:
    """A collective raised (gloo reports a closed peer connection at once;
    RCCL would block instead): if a peer died, this rank's heartbeat watchdog
    names it within its timeout and exits with EXIT_PEER_LOST -- the code the
    driver treats as a survivor's.  Waits for that verdict; returns (and the
    caller re-raises, a genuine failure of this rank) if no peer went silent."""
    from metisfl_amd.utils.metis_logger import MetisLogger
    MetisLogger.warning("collective call failed; waiting up to %.0f s for the heartbeat watchdog",
                        wd.timeout + 3 * wd.interval)
    end = time.time() + wd.timeout + 3 * wd.interval + 1.0
    while time.time() < end:
        time.sleep(0.1)  # the watchdog thread os._exit()s on a lost peer


def main(argv=None) -> int:
    ctx: dict = {}
    try:
        return _main(argv, ctx)
    except Exception:
        if ctx.get("wd") is not None:
            _await_peer_verdict(ctx["wd"])
        raise


def _main(argv, ctx: dict) -> int:
    argv = argv if argv is not None else sys.argv[1:]
    with open(argv[0]) as f:
        job = json.load(f)
    import torch

    from metisfl_amd.learner.learner import resolve_dataset
    from metisfl_amd.ops.optim import OptimizerSpec
    from metisfl_amd.parallel.comm import Comm
    from metisfl_amd.parallel.engine_bridge import RemoteCollectiveController
    from metisfl_amd.parallel.federation import CollectiveFederation, FederationConfig
    from metisfl_amd.parallel.watchdog import RankWatchdog
    from metisfl_amd.proto import metis_pb2, model_pb2
    from metisfl_amd.utils.grpc_controller_client import GRPCControllerClient

    comm = Comm(backend=job.get("backend"))
    rank = comm.rank
    # "ranks": the learners each process hosts (learners sharing a device are
    # co-located in one process: RCCL runs one rank per GPU); default one each
    ranks = job.get("ranks") or [[i] for i in range(len(job["learners"]))]
    if comm.world != len(ranks):
        raise RuntimeError(f"WORLD_SIZE {comm.world} != {len(ranks)} ranks in the job")
    mine = [job["learners"][i] for i in ranks[rank]]
    lcfg = mine[0]
    torch.manual_seed(job.get("seed", 0) + rank)
    opt = OptimizerSpec.from_proto(model_pb2.OptimizerConfig.FromString(bytes.fromhex(job["optimizer_hex"])))
    model_def = _load_model_def(job)
    train_recipe, test_recipe = _load_recipe(job.get("train_recipe")), _load_recipe(job.get("test_recipe"))
    nets, train_dss, test_dss = [], [], []
    if comm.device.type == "cuda":
        from metisfl_amd.models.colocated import configure_regime
        configure_regime(len(mine))  # this rank's co-located learners, before their models are built
    for lc in mine:
        n_ = model_def.get_model(batch_size=job["batch_size"], device=comm.device, optimizer=opt,
                                 seed=job.get("seed", 0))
        train = resolve_dataset(train_recipe, lc.get("train_path"))
        test = resolve_dataset(test_recipe, lc.get("test_path"))
        nets.append(n_)
        train_dss.append(n_.make_dataset(train.get_x(), train.get_y(), seed=lc.get("seed", rank)))
        test_dss.append(n_.make_dataset(test.get_x(), test.get_y(), seed=lc.get("seed", rank), shuffle=False)
                        if test is not None else None)
    net, train_ds, test_ds = nets[0], train_dss[0], test_dss[0]
    learner_ids = [l.get("id", f"learner_{i}") for i, l in enumerate(job["learners"])]
    fcfg = FederationConfig(**job["federation"])
    term = job.get("termination") or {}
    rounds = int(job["rounds"])
    cutoff_s = float(term["cutoff_mins"]) * 60.0 if term.get("cutoff_mins") else None
    metric, metric_cutoff = term.get("metric"), term.get("metric_cutoff")
    fault = job.get("fault") or {}
    ckpt_dir, every = job.get("checkpoint_dir"), int(job.get("checkpoint_every", 1) or 0)
    entity = metis_pb2.ServerEntity.FromString(bytes.fromhex(job["controller_hex"]))
    wd = None
    if comm.world > 1 and job.get("watchdog", True):
        wd = RankWatchdog(comm, interval_s=float(job.get("heartbeat_s", 1.0)),
                          timeout_s=float(job.get("heartbeat_timeout_s", 20.0))).start()
    ctx["wd"] = wd
    t_start = time.time()

    def initial_model(fed_load):
        if rank != 0 or job.get("resume_dir"):
            return
        client = GRPCControllerClient(entity, max_workers=1)
        try:
            lin = client.get_community_model_lineage(1)
            if len(lin.federated_models):
                fed_load(lin.federated_models[-1])
        finally:
            client.shutdown()

    endpoints = [(l["hostname"], l["port"]) for l in job["learners"]]
    if fcfg.protocol == "asynchronous":
        # every learner is its own FedRec participant, whatever its placement:
        # the ones this rank hosts run concurrently on their own streams
        from metisfl_amd.parallel.async_federation import AsyncCollectiveFederation
        from metisfl_amd.parallel.federation import install_community_model
        initial_model(lambda fm: install_community_model(net, fm, _he_decoder(fcfg, comm.device)))
        owners = [0] * len(job["learners"])
        for r, idx in enumerate(ranks):
            for i in idx:
                owners[i] = r
        gids = list(ranks[rank])
        # per-learner dataset sizes, in the job's learner order (the
        # controller's scaling inputs): every rank fills its learners' slots
        sz = torch.zeros(len(owners), dtype=torch.float64, device=comm.device)
        for g, d in zip(gids, train_dss):
            sz[g] = float(d.n)
        sizes = comm.all_gather_rows(sz).sum(0).cpu().numpy()
        engine = RemoteCollectiveController(entity, [int(x) for x in sizes], endpoints) if rank == 0 else None
        fed = AsyncCollectiveFederation(comm, nets, train_dss, fcfg, test_ds=test_dss, engine=engine,
                                        broadcast_initial=True, gids=gids, owners=owners, learner_ids=learner_ids)
        if job.get("resume_dir"):
            fed.resume(job["resume_dir"])
            if rank == 0:
                print(f"[collective-async] resumed at version {fed.version} on {len(owners)} learners "
                      f"(dropped learners {getattr(fed, 'resumed', {}).get('dropped')})", flush=True)
        delay = float((fcfg.extra or {}).get("debug_delay_s", {}).get(str(rank), 0.0))
        my_fault = fault if fault and int(fault.get("rank", -1)) == rank else None
        ups = fed.run_until(max_updates=rounds, cutoff_s=cutoff_s, metric=metric, metric_cutoff=metric_cutoff,
                            debug_delay_s=delay, checkpoint_dir=ckpt_dir, checkpoint_every=every,
                            fault_task=int(my_fault["round"]) if my_fault else None,
                            on_fault=lambda t: _inject_fault(rank, t, my_fault))
        if rank == 0:
            how = "secure PWA over ciphertexts" if fed.secure else "FedRec"
            print(f"[collective-async] {len(ups)} FedRec updates over {len(owners)} learners on {comm.world} "
                  f"ranks ({how}), stop: {fed.stop_reason}, staleness {[u.staleness for u in ups]}", flush=True)
            engine.close()
        if wd is not None:
            wd.stop()
        comm.close()
        return 0

    fed = CollectiveFederation(comm, nets, train_dss, fcfg, test_ds=test_dss, learner_ids=learner_ids,
                               broadcast_initial=False)
    initial_model(fed.load_community_model)
    if rank == 0:
        fed.engine = RemoteCollectiveController(entity, fed.dataset_sizes, endpoints)
    fed.broadcast_initial_model()
    if job.get("resume_dir"):
        fed.resume(job["resume_dir"], prev_rank=lcfg.get("prev_rank"))
        if rank == 0:
            print(f"[collective] resumed at round {fed.global_iteration} on {fed.n_learners} learners "
                  f"(checkpoint of {fed.resumed_from_learners})", flush=True)
    while fed.global_iteration < rounds:
        if fault and int(fault.get("rank", -1)) == rank and fed.global_iteration + 1 == int(fault.get("round", 0)):
            fed.flush_checkpoints()
            _inject_fault(rank, fed.global_iteration + 1, fault)
        rec = fed.run_round()
        if rank == 0:
            print(f"[collective] round {rec.global_iteration}: {rec.round_ms:.1f} ms "
                  f"(train {rec.train_ms:.1f}, aggregate {rec.aggregation_ms:.2f}, community eval "
                  f"{rec.community_eval_ms:.1f}) weights {rec.weights}", flush=True)
        if ckpt_dir and every and fed.global_iteration % every == 0 and fed.global_iteration < rounds:
            # staged device-to-device now, written while the next round trains
            rec.checkpoint_ms = fed.save_checkpoint(ckpt_dir, block=False)
            if rank == 0:
                print(f"[collective] checkpoint of round {rec.global_iteration} staged in "
                      f"{rec.checkpoint_ms:.1f} ms", flush=True)
        action = 0
        if rank == 0:
            m = fed.community_metric(rec, metric) if metric else None
            stop = (fed.stop_requested or (metric_cutoff is not None and m is not None and m >= float(metric_cutoff))
                    or (cutoff_s is not None and time.time() - t_start > cutoff_s))
            action = 1 if stop else (2 if fed.regroup_requested and fed.global_iteration < rounds else 0)
        action = _decision(comm, action)
        if action == 2:
            # a learner joins: a complete checkpoint of this round, then every
            # rank leaves; the driver relaunches the larger membership from it
            fed.save_checkpoint(ckpt_dir)
            fed.flush_checkpoints()
            if rank == 0:
                print(f"[collective] regroup after round {fed.global_iteration}: checkpointed, exiting for the "
                      f"relaunch", flush=True)
                fed.engine.close()
            if wd is not None:
                wd.stop()
            comm.close()
            return EXIT_REGROUP
        if action == 1:
            break
    if ckpt_dir:
        fed.save_checkpoint(ckpt_dir)  # the final one, complete before the ranks leave
    fed.flush_checkpoints()
    if rank == 0:
        st = net.state
        vals = st.to_numpy()
        fed.engine.snapshot_community([s.name for s in st.specs], [vals[s.name] for s in st.specs],
                                      [s.trainable for s in st.specs], fed.global_iteration)
        fed.engine.close()
    if wd is not None:
        wd.stop()
    comm.close()
    return 0


if __name__ == "__main__":
    from metisfl_amd.utils.launch import exit_process
    exit_process(main())  # no interpreter finalisation behind live c10d threads (utils/launch.py)
