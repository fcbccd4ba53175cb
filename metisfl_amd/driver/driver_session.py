"""Federation driver (reference: metisfl/driver/driver_session.py:29-585,
``DriverSessionBase`` / ``DriverSession``; same public methods).

Lifecycle: ``initialize_federation`` starts the controller, waits for its
health check, ships the initial community model (ReplaceCommunityModel), then
starts one learner per configured learner (0.1 s stagger);
``monitor_federation`` polls the controller for the termination signals
(rounds / metric cutoff / wall clock); ``shutdown_federation`` collects the
statistics (the reference's four keys) and stops everything.

MI355X-first differences:
  * learners are launched as LOCAL processes, one per GPU, pinned with
    HIP_VISIBLE_DEVICES (the reference SSHes even to localhost with fabric,
    which is not installed); ``Launcher: ssh`` runs the same command lines
    through the ``ssh`` CLI for remote hosts;
  * the model is shipped as a small JSON definition of a built-in family
    (or a cloudpickled TorchModelDef), not a tarred SavedModel;
  * the on-node data plane (RCCL all-reduce instead of gRPC model
    transfer) is ``DriverSession.run_collective`` below: one learner process
    per GPU under one process group, rank 0 reporting rounds to the
    controller.
"""
from __future__ import annotations

import json
import os
import shlex
import shutil
import socket
import subprocess
import time

from google.protobuf.json_format import MessageToDict

from metisfl_amd.models.model_def import StaticModelDef, TorchModelDef
from metisfl_amd.utils import fedenv_parser
from metisfl_amd.utils.grpc_controller_client import GRPCControllerClient
from metisfl_amd.utils.grpc_learner_client import GRPCLearnerClient
from metisfl_amd.utils.init_services_factory import MetisInitServicesCmdFactory
from metisfl_amd.utils.metis_logger import MetisASCIIArt, MetisLogger
from metisfl_amd.utils.proto_messages_factory import MetisProtoMessages as M
from metisfl_amd.utils.proto_messages_factory import ModelProtoMessages as MM
from metisfl_amd.utils.ssl_configurator import SSLConfigurator
from metisfl_amd.utils.tensor_codec import model_from_arrays


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _ssl_pb(enable: bool, cfg):
    if not enable:
        return M.construct_ssl_config_pb(False)
    if cfg is not None and cfg.public_certificate_file:
        return M.construct_ssl_config_pb(True, M.construct_ssl_config_files_pb(cfg.public_certificate_file,
                                                                            cfg.private_key_file))
    return SSLConfigurator.default_ssl_config_pb()


class DriverSessionBase:

    def __init__(self, fed_env, model, train_dataset_recipe_fn, validation_dataset_recipe_fn=None,
                 test_dataset_recipe_fn=None, working_dir: str = "/tmp/metis_amd/", device: str | None = None,
                 seed: int = 0, fake_train_delay: float = 0.0, collective_options: dict | None = None):
        MetisASCIIArt.print()
        self.federation_environment = fed_env if isinstance(fed_env, fedenv_parser.FederationEnvironment) \
            else fedenv_parser.FederationEnvironment(fed_env)
        env = self.federation_environment
        self.num_participating_learners = len(env.learners)
        self.working_dir = working_dir
        if os.path.exists(working_dir):
            shutil.rmtree(working_dir)
        os.makedirs(working_dir)
        self.device = device
        self.seed = seed
        # collective data plane knobs: checkpoint_every (rounds, default 5;
        # written in the background), max_recoveries (lost-rank relaunches,
        # default 2), heartbeat_timeout_s, fault ({"rank", "round"[, "signal":
        # "KILL"]}: fault injection for tests), extra
        # (FederationConfig.extra: test hooks such as uneven learner delays)
        self.collective_options = dict(collective_options or {})
        self.recoveries: list[dict] = []
        self.regroups: list[dict] = []      # learners admitted into a running collective federation
        self._pending_joins: list = []
        self.fake_train_delay = fake_train_delay  # echo learners only
        self._model_dir = os.path.join(working_dir, "model_definition")
        self.neural_engine = self._save_model(model)
        if train_dataset_recipe_fn is None:
            raise RuntimeError("Train dataset recipe cannot be empty.")
        self.train_dataset_recipe_fp = self._dump_recipe(train_dataset_recipe_fn, "model_train_dataset_ops.pkl")
        self.validation_dataset_recipe_fp = self._dump_recipe(validation_dataset_recipe_fn,
                                                              "model_validation_dataset_ops.pkl")
        self.test_dataset_recipe_fp = self._dump_recipe(test_dataset_recipe_fn, "model_test_dataset_ops.pkl")
        self.enable_ssl = env.communication_protocol.enable_ssl
        self._controller_entity = M.construct_server_entity_pb(
            env.controller.grpc_servicer.hostname, env.controller.grpc_servicer.port,
            _ssl_pb(self.enable_ssl, env.controller.ssl_configs))
        self._learner_entities = {
            l.learner_id: M.construct_server_entity_pb(l.grpc_servicer.hostname, l.grpc_servicer.port,
                                                       _ssl_pb(self.enable_ssl, l.ssl_configs))
            for l in env.learners}
        self._driver_controller_grpc_client = GRPCControllerClient(self._controller_entity, max_workers=1)
        self._driver_learner_grpc_clients = {lid: GRPCLearnerClient(e) for lid, e in self._learner_entities.items()}
        self._federation_statistics: dict = {}
        self._procs: dict[str, subprocess.Popen] = {}
        self._init_he(env)
        self._cmds = MetisInitServicesCmdFactory()

    # -- setup helpers -----------------------------------------------------------------
    def _save_model(self, model) -> str:
        if model == "fake" or model is None:  # echo learners: orchestration only
            self._initial_model = model_from_arrays(["w"], [__import__("numpy").zeros(4, "float32")])
            return "fake"
        if isinstance(model, str):
            model = StaticModelDef(model)
        if isinstance(model, StaticModelDef):
            model.save(self._model_dir)
            net = model.get_model(batch_size=1, device="cpu", seed=self.seed)
            st = net.state
            vals = st.to_numpy()
            self._initial_model = model_from_arrays([s.name for s in st.specs], [vals[s.name] for s in st.specs],
                                                    [s.trainable for s in st.specs])
            return "static"
        if isinstance(model, TorchModelDef):
            import cloudpickle
            import inspect
            os.makedirs(self._model_dir, exist_ok=True)
            mod = inspect.getmodule(type(model))
            if mod is not None and mod.__name__ not in ("__main__",):
                cloudpickle.register_pickle_by_value(mod)
            with open(os.path.join(self._model_dir, "model_def.pkl"), "wb") as f:
                cloudpickle.dump(model, f)
            from metisfl_amd.models.torch_ops import TorchModelOps
            names, trainable, values = TorchModelOps(model, device="cpu", seed=self.seed).get_model_weights()
            self._initial_model = model_from_arrays(names, values, trainable)
            return "torch"
        raise RuntimeError("Not a supported model type (StaticModelDef, family name or TorchModelDef).")

    def _dump_recipe(self, fn, name):
        if fn is None:
            return None
        import cloudpickle
        p = os.path.join(self.working_dir, name)
        with open(p, "wb") as f:
            cloudpickle.dump(fn, f)
        return p

    def _init_he(self, env):
        he = env.homomorphic_encryption
        self._he_scheme = None
        if he is not None and he.scheme.upper() == "CKKS":
            from metisfl_amd import _engine
            d = os.path.join(self.working_dir, "cryptoparams")
            os.makedirs(d, exist_ok=True)
            self._he_scheme = _engine.CKKS(he.batch_size, he.scaling_factor_bits)
            self._he_scheme.gen_crypto_context_and_keys(d)
            files = self._he_scheme.get_crypto_params_files()
            ckks = M.construct_ckks_scheme_config_pb(he.batch_size, he.scaling_factor_bits)
            self._controller_he_scheme_config_pb = M.construct_he_scheme_config_pb(
                enabled=True, crypto_context_file=files["crypto_context_file"], ckks_scheme_config_pb=ckks)
            self._learners_he_scheme_config_pb = M.construct_he_scheme_config_pb(
                enabled=True, crypto_context_file=files["crypto_context_file"],
                public_key_file=files["public_key_file"], private_key_file=files["private_key_file"],
                ckks_scheme_config_pb=ckks)
        else:
            self._controller_he_scheme_config_pb = M.construct_he_scheme_config_pb(enabled=False)
            self._learners_he_scheme_config_pb = M.construct_he_scheme_config_pb(enabled=False)

    # -- service command lines ---------------------------------------------------------------
    def _controller_params(self):
        env = self.federation_environment
        rule = env.global_model_config.aggregation_rule
        agg = M.construct_aggregation_rule_pb(rule.aggregation_rule_name, rule.aggregation_rule_scaling_factor,
                                              rule.aggregation_rule_stride_length,
                                              self._controller_he_scheme_config_pb)
        gms = M.construct_global_model_specs(agg, env.global_model_config.participation_ratio)
        cp = env.communication_protocol
        cs = M.construct_communication_specs_pb(cp.name, cp.semi_synchronous_lambda, cp.semi_sync_recompute_num_updates)
        lm = env.local_model_config
        opt = MM.construct_optimizer_config_pb_from_kwargs(lm.optimizer_config.optimizer_pb_kwargs)
        mh = M.construct_controller_modelhyperparams_pb(lm.batch_size, lm.local_epochs, opt,
                                                        lm.validation_percentage)
        ms = env.model_store_config
        store = M.construct_model_store_config_pb(ms.name, ms.eviction_policy, ms.eviction_lineage_length,
                                                  ms.connection_configs.hostname, ms.connection_configs.port)
        return gms, cs, mh, store

    def _init_controller_cmd(self):
        gms, cs, mh, store = self._controller_params()
        return self._cmds.init_controller_target(self._controller_entity, gms, cs, mh, store)

    def _init_learner_cmd(self, learner_instance, controller_instance=None):
        lid = learner_instance.learner_id
        dc = learner_instance.dataset_configs
        dev = self.device
        if dev is None:
            dev = "cuda" if learner_instance.devices else None
        return self._cmds.init_learner_target(
            self._learner_entities[lid], self._controller_entity, self._learners_he_scheme_config_pb,
            self._model_dir, dc.train_dataset_path, dc.validation_dataset_path, dc.test_dataset_path,
            self.train_dataset_recipe_fp, self.validation_dataset_recipe_fp, self.test_dataset_recipe_fp,
            neural_engine=self.neural_engine, device=dev,
            credentials_dir=os.path.join(self.working_dir, f"learner_{learner_instance.grpc_servicer.port}_credentials"),
            seed=self.seed, fake_train_delay=self.fake_train_delay)

    # -- process control -----------------------------------------------------------------------
    def _spawn(self, name, cmd, env_extra=None, remote=None):
        log = open(os.path.join(self.working_dir, f"{name}.log"), "w")
        env = dict(os.environ)
        env.update(env_extra or {})
        root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        env["PYTHONPATH"] = root + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
        if remote is not None:  # Launcher: ssh
            cc = remote.connection_configs
            exports = " ".join(f"{k}={shlex.quote(v)}" for k, v in (env_extra or {}).items())
            remote_cmd = f"{cc.on_login.rstrip(';') + ' && ' if cc.on_login else ''}cd {remote.project_home or '.'} " \
                         f"&& {exports} {' '.join(shlex.quote(c) for c in cmd)}"
            target = f"{cc.username}@{cc.hostname}" if cc.username else cc.hostname
            cmd = ["ssh"] + (["-p", str(cc.port)] if cc.port else []) + \
                (["-i", cc.key_filename] if cc.key_filename else []) + [target, remote_cmd]
        self._procs[name] = subprocess.Popen(cmd, stdout=log, stderr=subprocess.STDOUT, env=env)
        return self._procs[name]

    def _init_controller(self):
        ssh = self.federation_environment.launcher == "ssh"
        return self._spawn("controller", self._init_controller_cmd(),
                           remote=self.federation_environment.controller if ssh else None)

    def _init_learner(self, learner_instance, controller_instance=None):
        extra = {}
        if learner_instance.devices:
            extra["HIP_VISIBLE_DEVICES"] = ",".join(str(d) for d in learner_instance.devices)
        ssh = self.federation_environment.launcher == "ssh"
        if not ssh and not learner_instance.devices:  # host-CPU learners of this machine share its cores
            extra.update(self._cpu_share(len(self.federation_environment.learners)))
        return self._spawn(f"learner_{learner_instance.learner_id}",
                           self._init_learner_cmd(learner_instance, controller_instance), extra,
                           remote=learner_instance if ssh else None)

    def _ship_model_to_controller(self):
        model = self._initial_model
        if self._he_scheme is not None:
            from metisfl_amd.utils.tensor_codec import model_to_arrays
            names, arrays, tr = model_to_arrays(model)
            self._he_scheme.load_crypto_context_from_file(self._he_scheme.get_crypto_params_files()["crypto_context_file"])
            model = model_from_arrays(names, arrays, tr, self._he_scheme)
        return self._driver_controller_grpc_client.replace_community_model(1, model, request_retries=3)

    # -- on-node collective data plane (DataPlane: rccl) ----------------------------------------
    @property
    def collective(self) -> bool:
        return self.federation_environment.data_plane == "rccl"

    _RULES = {"FEDAVG": "fed_avg", "FEDSTRIDE": "fed_stride", "FEDREC": "fed_rec", "PWA": "fed_avg"}

    def _collective_federation(self) -> dict:
        """FederationConfig of the collective ranks from the YAML: protocol,
        aggregation rule, scaling factor, stride, semi-sync knobs, secure
        aggregation.  Combinations the collective data plane does not run
        raise instead of silently falling back to synchronous FedAvg."""
        env = self.federation_environment
        lm, cp = env.local_model_config, env.communication_protocol
        rule = env.global_model_config.aggregation_rule
        rname = (rule.aggregation_rule_name or "FedAvg").upper()
        if rname not in self._RULES:
            raise RuntimeError(f"aggregation rule {rule.aggregation_rule_name!r} is not supported on DataPlane: rccl")
        if cp.is_asynchronous:
            protocol = "asynchronous"  # with CKKS: PWA over the learners' latest ciphertexts (AsyncPWA)
        elif cp.is_semi_synchronous:
            protocol = "semi_synchronous"
        elif cp.is_synchronous:
            protocol = "synchronous"
        else:
            raise RuntimeError(f"unknown communication protocol {cp.name!r}")
        return {"protocol": protocol, "aggregation": self._RULES[rname],
                "stride_length": int(rule.aggregation_rule_stride_length or 0),
                "scaling_factor": {"NumTrainingExamples": "NUM_TRAINING_EXAMPLES",
                                   "NumCompletedBatches": "NUM_COMPLETED_BATCHES",
                                   "NumParticipants": "NUM_PARTICIPANTS"}.get(
                    rule.aggregation_rule_scaling_factor or "NumTrainingExamples", "NUM_TRAINING_EXAMPLES"),
                "batch_size": lm.batch_size, "local_epochs": lm.local_epochs,
                "semi_sync_lambda": float(cp.semi_synchronous_lambda or 2.0),
                "semi_sync_recompute": bool(cp.semi_sync_recompute_num_updates),
                "participation_ratio": float(env.global_model_config.participation_ratio or 1.0),
                "secure_aggregation": self._he_scheme is not None,
                **self._collective_he(),
                "extra": dict(self.collective_options.get("extra", {}))}

    def _collective_he(self) -> dict:
        """The driver's CKKS parameters and key files for the collective ranks
        (the reference's learners load the driver's key pair,
        driver_session.py:122-135)."""
        if self._he_scheme is None:
            return {}
        he = self.federation_environment.homomorphic_encryption
        files = self._he_scheme.get_crypto_params_files()
        return {"he_batch_size": int(he.batch_size), "he_scaling_bits": int(he.scaling_factor_bits),
                "he_key_dir": os.path.dirname(files["crypto_context_file"])}

    def _collective_job(self, rounds: int, learners=None, resume_dir: str | None = None,
                        prev_ranks: list[int] | None = None, fault: dict | None = None, tag: str = "",
                        ranks: list[list[int]] | None = None) -> str:
        """The JSON job description every collective rank reads (``learners``
        in rank order, ``ranks``: the learner indices each process hosts)."""
        env = self.federation_environment
        lm = env.local_model_config
        if self.neural_engine not in ("static", "torch"):
            raise RuntimeError("the collective data plane runs StaticModelDef / TorchModelDef models")
        learners = list(env.learners) if learners is None else learners
        opt = MM.construct_optimizer_config_pb_from_kwargs(lm.optimizer_config.optimizer_pb_kwargs)
        ts = env.termination_signals
        o = self.collective_options
        job = {"model_dir": self._model_dir, "model_kind": self.neural_engine,
               "batch_size": lm.batch_size, "seed": self.seed,
               "optimizer_hex": opt.SerializeToString().hex(),
               "controller_hex": self._controller_entity.SerializeToString().hex(),
               "train_recipe": self.train_dataset_recipe_fp, "test_recipe": self.test_dataset_recipe_fp,
               "rounds": rounds, "federation": self._collective_federation(),
               "termination": {"cutoff_mins": ts.execution_time_cutoff_mins, "metric": env.evaluation_metric,
                               "metric_cutoff": ts.metric_cutoff_score},
               "checkpoint_dir": os.path.join(self.working_dir, "collective_checkpoint"),
               # staged on the device and written in the background (parallel/
               # checkpoint.py); every 5 rounds by default, plus the last one
               "checkpoint_every": int(o.get("checkpoint_every", 5)),
               "heartbeat_timeout_s": float(o.get("heartbeat_timeout_s", 20.0)),
               "resume_dir": resume_dir, "fault": fault,
               "backend": "gloo" if self.device == "cpu" else None,
               "learners": [{"id": l.learner_id, "hostname": l.grpc_servicer.hostname or "localhost",
                             "port": int(l.grpc_servicer.port or 0) or 1 + self._learner_index(l),
                             "train_path": l.dataset_configs.train_dataset_path,
                             "test_path": l.dataset_configs.test_dataset_path, "devices": l.devices,
                             "seed": self._learner_index(l),
                             "prev_rank": prev_ranks[i] if prev_ranks is not None else None}
                            for i, l in enumerate(learners)],
               "ranks": ranks or [[i] for i in range(len(learners))]}
        p = os.path.join(self.working_dir, f"collective_job{tag}.json")
        with open(p, "w") as f:
            json.dump(job, f)
        return p

    def _learner_index(self, learner) -> int:
        return [l.learner_id for l in self.federation_environment.learners].index(learner.learner_id)

    @staticmethod
    def _device_groups(learners) -> list[list]:
        """Learners that name the same device(s) share one process: RCCL runs
        one rank per GPU, and co-located learners train concurrently on their
        own HIP streams (models/colocated.py) -- the reference's 10 learners
        on 5 GPUs (examples/config/cifar10/...momentumsgd.yaml) become 5 ranks
        of 2.  Learners without devices get a process each."""
        groups: dict = {}
        for i, l in enumerate(learners):
            key = tuple(l.devices) if l.devices else ("solo", i)
            groups.setdefault(key, []).append(l)
        return list(groups.values())

    def _init_collective_learners(self, rounds: int, learners=None, resume_dir=None, prev_ranks=None,
                                  fault=None, tag: str = ""):
        """One process per device (hosting that device's learners) under one
        process group; the torch.distributed env is set here, before any of
        them touches a GPU (reference counterpart: driver_session.py:529-582).
        Each launch is a set of FRESH processes (never a re-exec of one that
        touched the GPU)."""
        import sys
        learners = list(self.federation_environment.learners) if learners is None else learners
        groups = self._device_groups(learners)
        flat = [l for g in groups for l in g]  # rank order
        if prev_ranks is not None:  # legacy per-rank checkpoints: follow the learners into rank order
            by_id = {l.learner_id: pr for l, pr in zip(learners, prev_ranks)}
            prev_ranks = [by_id[l.learner_id] for l in flat]
        ranks, k = [], 0
        for g in groups:
            ranks.append(list(range(k, k + len(g))))
            k += len(g)
        job = self._collective_job(rounds, flat, resume_dir, prev_ranks, fault, tag, ranks)
        port = free_port()
        self._collective_members = flat
        self._collective_groups = groups
        for rank, g in enumerate(groups):
            l = g[0]
            extra = {"RANK": str(rank), "WORLD_SIZE": str(len(groups)), "MASTER_ADDR": "127.0.0.1",
                     "MASTER_PORT": str(port), "HSA_ENABLE_IPC_MODE_LEGACY": "0",
                     "LOCAL_RANK": str(l.devices[0] if l.devices else rank)}
            extra["METISFL_WATCHDOG_REPORT_DIR"] = self._watchdog_dir(tag)
            if self.device == "cpu":
                extra.update(CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
                extra.update(self._cpu_share(len(groups)))
            self._spawn(self._proc_name(g), [sys.executable, "-m", "metisfl_amd.learner.collective", job], extra)
        self._collective_tag = tag

    @staticmethod
    def _cpu_share(n_procs: int) -> dict:
        """CPU ranks on one host split its cores: n processes each starting one
        OpenMP thread per core oversubscribe n-fold, and spin-waiting barriers
        make that far slower than n-fold.  A user's OMP_NUM_THREADS wins."""
        if "OMP_NUM_THREADS" in os.environ:
            return {}
        return {"OMP_NUM_THREADS": str(max(1, (os.cpu_count() or 1) // max(1, n_procs)))}

    @staticmethod
    def _proc_name(group) -> str:
        """A collective process is named (and logs) after the first learner it hosts."""
        return f"learner_{group[0].learner_id}"

    def _watchdog_dir(self, tag: str) -> str:
        return os.path.join(self.working_dir, f"watchdog{tag}")

    # a rank that lost a peer exits with this code (parallel/watchdog.py)
    _PEER_EXIT = 75

    def _recover_collective(self, failed_name: str, code: int) -> None:
        """A collective rank died: stop the survivors (blocked in a collective,
        or already out on their watchdog), and relaunch them as fresh
        processes on the smaller world from the last FederatedModel checkpoint
        (the reference's learners may leave at any time,
        controller.cc:171-199).

        Which ranks failed is decided from the exit codes seen BEFORE the
        driver signals anyone: a rank that had already exited with anything
        but 0 or the watchdog's peer-loss code (including -9 / -15 from a
        signal the driver did not send, e.g. the OOM killer) is a failure;
        ranks the driver terminates here are survivors."""
        members = list(self._collective_members)
        groups = list(getattr(self, "_collective_groups", [[l] for l in members]))
        names = {self._proc_name(g): g for g in groups}
        before = {n: self._procs[n].poll() for n in names if n in self._procs}
        before[failed_name] = code
        # give ranks that are on their way out (watchdog exit) a moment, so a
        # peer-loss exit is not mistaken for a rank the driver had to stop
        end = time.time() + float(self.collective_options.get("recovery_grace_s", 3.0))
        while time.time() < end and any(self._procs[n].poll() is None for n in before if before[n] is None):
            time.sleep(0.05)
        for n in before:
            if before[n] is None:
                before[n] = self._procs[n].poll()
        signalled = set()
        for name, p in self._procs.items():
            if name in names and p.poll() is None:
                p.terminate()
                signalled.add(name)
        for name, p in self._procs.items():
            if name in names:
                try:
                    p.wait(timeout=30)
                except subprocess.TimeoutExpired:
                    p.kill()
                    p.wait(10)
        # a rank that left for a regroup (checkpointed, EXIT_REGROUP) is healthy too
        failed = {n for n, rc in before.items()
                  if n not in signalled and rc not in (None, 0, self._PEER_EXIT, self.EXIT_REGROUP)}
        # a hung rank does not exit: the survivors' watchdogs name it
        order = [self._proc_name(g) for g in groups]
        wdir = self._watchdog_dir(getattr(self, "_collective_tag", ""))
        if os.path.isdir(wdir):
            for fn in os.listdir(wdir):
                try:
                    with open(os.path.join(wdir, fn)) as f:
                        peer = int(json.load(f)["peer"])
                except (OSError, ValueError, KeyError):
                    continue
                if 0 <= peer < len(order) and order[peer] in signalled:
                    failed.add(order[peer])
        if not failed:
            raise RuntimeError(f"collective learners left on a lost peer, but the failed rank is unknown "
                               f"({failed_name} exited with {code})")
        survivors = [l for n, g in names.items() if n not in failed for l in g]
        if not survivors:
            raise RuntimeError(f"every collective learner failed ({failed_name} exited with {code})")
        from metisfl_amd.parallel import checkpoint as ck
        ckpt = os.path.join(self.working_dir, "collective_checkpoint")
        found = ck.resolve(ckpt)
        resume = ckpt if found else None
        rank_of = {l.learner_id: r for r, g in enumerate(groups) for l in g}
        prev = [rank_of[l.learner_id] for l in survivors]
        gi = None
        if found:
            with open(os.path.join(found, "federation.json")) as f:
                gi = json.load(f)["global_iteration"]
        self.recoveries.append({"failed": sorted(failed), "exit_code": code, "survivors": len(survivors),
                                "lost_learners": sorted(l.learner_id for n in failed for l in names[n]),
                                "resumed_from_round": gi, "at": time.time()})
        MetisLogger.warning("collective learner(s) %s lost (exit %d): relaunching %d survivors from round %s",
                            sorted(failed), code, len(survivors), gi)
        for n in names:
            log = os.path.join(self.working_dir, f"{n}.log")
            if os.path.exists(log):
                os.replace(log, log + f".attempt{len(self.recoveries)}")
            self._procs.pop(n, None)
        self._init_collective_learners(self.federation_environment.termination_signals.federation_rounds,
                                       survivors, resume, prev, None, tag=f"_r{len(self.recoveries)}")

    # -- learners joining a running collective federation ---------------------------------------------
    EXIT_REGROUP = 76  # learner/collective.py: checkpointed for a relaunch on a new membership

    def join_collective_learner(self, learner) -> None:
        """Admit a learner into a RUNNING collective (DataPlane: rccl)
        federation -- the reference's JoinFederation / AddLearner, which
        registers the joiner and schedules it right away
        (controller.cc:98-168).  The collective ranks finish their current
        round, write a complete checkpoint and exit (EXIT_REGROUP);
        ``monitor_federation`` relaunches the larger membership from it as
        fresh processes: the newcomer starts from the community model with a
        fresh optimizer state, the step budgets and FedAvg weights are
        recomputed over the new shards, and the round count continues.
        ``learner``: a ``fedenv_parser.Learner`` or its YAML mapping."""
        from metisfl_amd.controller import collective_service as cs
        from metisfl_amd.utils.fedenv_parser import Learner
        from metisfl_amd.utils.grpc_services import make_channel
        if not self.collective:
            raise RuntimeError("join_collective_learner needs DataPlane: rccl (gRPC learners join by themselves)")
        if self.federation_environment.communication_protocol.is_asynchronous:
            # the asynchronous ranks never stop at a round boundary, so a
            # regroup would never be acted on
            raise RuntimeError("join_collective_learner: the asynchronous collective protocol does not regroup; "
                               "start the federation with every learner")
        if isinstance(learner, dict):
            learner = Learner(learner)
        self.federation_environment.learners.learners.append(learner)
        self._pending_joins.append(learner)
        ch = make_channel(self._controller_entity)
        try:
            cs.call(ch, "RequestRegroup", {}, timeout=30)
        finally:
            ch.close()
        MetisLogger.info("learner %s joins the collective federation at the next round boundary",
                         learner.learner_id)

    def _regroup_ready(self, timeout_s: float = 120.0) -> bool:
        """True when every collective rank left with EXIT_REGROUP (waits for
        the stragglers of a regroup that has started); False otherwise."""
        procs = {n: p for n, p in self._procs.items() if n.startswith("learner_")}
        if not any(p.poll() == self.EXIT_REGROUP for p in procs.values()):
            return False
        end = time.time() + timeout_s
        while time.time() < end and any(p.poll() is None for p in procs.values()):
            time.sleep(0.05)
        return all(p.poll() == self.EXIT_REGROUP for p in procs.values())

    def _regroup_collective(self) -> None:
        from metisfl_amd.parallel import checkpoint as ck
        old = list(self._collective_members)
        joins, self._pending_joins = list(self._pending_joins), []
        members = old + joins
        ckpt = os.path.join(self.working_dir, "collective_checkpoint")
        found = ck.resolve(ckpt)
        if found is None:
            raise RuntimeError("collective regroup: the ranks left no checkpoint")
        with open(os.path.join(found, "federation.json")) as f:
            gi = json.load(f)["global_iteration"]
        self.regroups.append({"joined": [l.learner_id for l in joins], "world": len(members),
                              "at_round": gi, "at": time.time()})
        MetisLogger.info("collective federation regroups at round %d: %d -> %d learners", gi, len(old), len(members))
        for g in getattr(self, "_collective_groups", [[l] for l in old]):
            n = self._proc_name(g)
            log = os.path.join(self.working_dir, f"{n}.log")
            if os.path.exists(log):
                os.replace(log, log + f".group{len(self.regroups)}")
            self._procs.pop(n, None)
        # old members keep their learner-local state (checkpoint files by learner id); joiners start fresh
        rank_of = {l.learner_id: r for r, g in enumerate(getattr(self, "_collective_groups", [[l] for l in old]))
                   for l in g}
        self._init_collective_learners(self.federation_environment.termination_signals.federation_rounds,
                                       members, ckpt, [rank_of.get(l.learner_id, -1) for l in members], None,
                                       tag=f"_g{len(self.regroups)}")

    # -- public API -----------------------------------------------------------------------------------
    def initialize_federation(self):
        if self.collective:
            self._collective_federation()  # unsupported combinations fail before anything starts
        self._init_controller()
        ok = self._driver_controller_grpc_client.check_health_status(request_retries=10, request_timeout=30)
        if not ok:
            raise RuntimeError("controller did not come up; see controller.log")
        self._ship_model_to_controller()
        if self.collective:
            self._init_collective_learners(self.federation_environment.termination_signals.federation_rounds,
                                           fault=self.collective_options.get("fault"))
            return
        for l in self.federation_environment.learners:
            self._init_learner(l, self.federation_environment.controller)
            time.sleep(0.1)

    def run_collective(self, request_every_secs: float = 1.0) -> dict:
        """Whole collective federation: controller up, one rank per GPU,
        wait for the configured rounds, statistics, shutdown."""
        if not self.collective:
            raise RuntimeError("run_collective needs DataPlane: rccl in the federation environment")
        self.initialize_federation()
        try:
            self.termination_reason = self.monitor_federation(request_every_secs)
        finally:
            self.shutdown_federation()
        return self.get_federation_statistics()

    def monitor_federation(self, request_every_secs: float = 10):
        env = self.federation_environment
        rounds = env.termination_signals.federation_rounds
        cp = env.communication_protocol
        cutoff_mins = env.termination_signals.execution_time_cutoff_mins
        metric_cutoff = env.termination_signals.metric_cutoff_score
        metric = env.evaluation_metric
        st = time.time()
        while True:
            time.sleep(request_every_secs)
            if self.collective and self._regroup_ready():
                self._regroup_collective()
                continue
            for name, p in list(self._procs.items()):
                if p.poll() is not None and p.returncode != 0:
                    if (self.collective and name.startswith("learner_")
                            and len(self.recoveries) < int(self.collective_options.get("max_recoveries", 2))):
                        self._recover_collective(name, p.returncode)
                        break
                    raise RuntimeError(f"{name} exited with {p.returncode}; see {name}.log")
            evals = self._driver_controller_grpc_client.get_community_model_evaluation_lineage(-1)
            for res in evals.community_evaluation:
                scores = [float(e.test_evaluation.metric_values[metric]) for e in res.evaluations.values()
                          if metric in e.test_evaluation.metric_values]
                if scores and sum(scores) / len(scores) >= metric_cutoff:
                    MetisLogger.info("Exceeded evaluation metric cutoff score. Exiting ...")
                    return "metric"
            if self.collective and all(p.poll() == 0 for n, p in self._procs.items() if n.startswith("learner_")):
                MetisLogger.info("Collective learners completed their rounds. Exiting ...")
                return "rounds"
            md = self._driver_controller_grpc_client.get_runtime_metadata(num_backtracks=0).metadata
            if (cp.is_synchronous or cp.is_semi_synchronous) and rounds and len(md) > 0:
                if max(m.global_iteration for m in md) > rounds:
                    MetisLogger.info("Exceeded federation rounds cutoff point. Exiting ...")
                    return "rounds"
            if (time.time() - st) / 60 > cutoff_mins:
                MetisLogger.info("Exceeded execution time cutoff minutes. Exiting ...")
                return "time"

    def _collect_local_statistics(self):
        c = self._driver_controller_grpc_client
        learners = c.get_participating_learners()
        ids = [l.id for l in learners.learner]
        self._federation_statistics["learners_descriptor"] = MessageToDict(learners, preserving_proto_field_name=True)
        self._federation_statistics["learners_models_results"] = MessageToDict(
            c.get_local_task_lineage(-1, ids), preserving_proto_field_name=True)

    def _collect_global_statistics(self):
        c = self._driver_controller_grpc_client
        self._federation_statistics["federation_runtime_metadata"] = MessageToDict(
            c.get_runtime_metadata(num_backtracks=0), preserving_proto_field_name=True)
        self._federation_statistics["community_model_results"] = MessageToDict(
            c.get_community_model_evaluation_lineage(-1), preserving_proto_field_name=True)

    def get_federation_statistics(self) -> dict:
        return self._federation_statistics

    def save_statistics(self, path: str) -> None:
        with open(path, "w") as f:
            json.dump(self._federation_statistics, f, indent=1)

    def _request_collective_stop(self) -> None:
        """Ask running collective ranks to leave after their current round."""
        from metisfl_amd.controller import collective_service as cs
        from metisfl_amd.utils.grpc_services import make_channel
        ch = make_channel(self._controller_entity)
        try:
            cs.call(ch, "RequestStop", {}, timeout=10)
        except Exception as e:  # noqa: BLE001 - the controller may already be gone
            MetisLogger.warning("collective stop request failed: %r", e)
        finally:
            ch.close()

    def shutdown_federation(self, timeout: float = 60):
        try:
            if self.collective and any(p.poll() is None for n, p in self._procs.items() if n.startswith("learner_")):
                self._request_collective_stop()
                end = time.time() + timeout
                for n, p in self._procs.items():
                    if n.startswith("learner_"):
                        try:
                            p.wait(timeout=max(0.1, end - time.time()))
                        except subprocess.TimeoutExpired:
                            pass
            self._collect_local_statistics()
            # collective learners have no gRPC server: they exit after their rounds
            for c in ([] if self.collective else self._driver_learner_grpc_clients.values()):
                try:
                    c.shutdown_learner(request_retries=1, request_timeout=30, block=True)
                except Exception as e:  # noqa: BLE001 - a dead learner must not block shutdown
                    MetisLogger.warning("learner shutdown failed: %r", e)
                c.shutdown()
            self._collect_global_statistics()
            self._driver_controller_grpc_client.shutdown_controller(request_retries=2, request_timeout=30)
            self._driver_controller_grpc_client.shutdown()
        finally:
            end = time.time() + timeout
            for name, p in self._procs.items():
                try:
                    p.wait(timeout=max(0.1, end - time.time()))
                except subprocess.TimeoutExpired:
                    MetisLogger.warning("%s did not exit; terminating pid %d", name, p.pid)
                    p.terminate()
                    p.wait(10)


class DriverSession(DriverSessionBase):
    """Same constructor as the reference DriverSession."""
