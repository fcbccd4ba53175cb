"""``FederationEnvironment`` YAML parser (reference:
metisfl/utils/fedenv_parser.py:4-309; same keys, same defaults).

Additions for this framework (all optional, ignored by reference configs):
  * ``Devices`` on a learner -- GPU ordinals (HIP); ``CudaDevices`` is still
    accepted and means the same;
  * ``Launcher`` -- "local" (default: subprocesses on this node, one per GPU)
    or "ssh" (remote hosts, the reference's fabric path);
  * ``NeuralEngine`` on LocalModelConfig -- "static" | "torch" | "fake".
ConnectionConfigs.Username is only required for the ssh launcher (the
reference always requires it because it always SSHes, even to localhost).
YAML is read with ``yaml.SafeLoader`` only."""
from __future__ import annotations

import yaml


def _get(m, k, default=None):
    return (m or {}).get(k, default)


class DockerImage:
    def __init__(self, docker_image):
        self.docker_image = docker_image


class TerminationSignals:
    def __init__(self, m):
        self.federation_rounds = _get(m, "FederationRounds", 100)
        self.execution_time_cutoff_mins = _get(m, "ExecutionCutoffTimeMins", 1e6) or 1e6
        self.metric_cutoff_score = _get(m, "MetricCutoffScore", 1)


class HomomorphicEncryption:
    def __init__(self, m):
        self.scheme = _get(m, "Scheme", "")
        self.batch_size = _get(m, "BatchSize")
        self.scaling_factor_bits = _get(m, "ScalingFactorBits")


class CommunicationProtocol:
    def __init__(self, m):
        self.enable_ssl = bool(_get(m, "EnableSSL", False))
        self.name = _get(m, "Name", "Synchronous")
        up = self.name.upper()
        self.is_asynchronous = up == "ASYNCHRONOUS"
        self.is_synchronous = up == "SYNCHRONOUS"
        self.is_semi_synchronous = up in ("SEMI_SYNCHRONOUS", "SEMISYNCHRONOUS")
        self.specifications = _get(m, "Specifications")
        self.semi_synchronous_lambda = self.semi_sync_recompute_num_updates = None
        if self.specifications and self.is_semi_synchronous:
            self.semi_synchronous_lambda = self.specifications.get("SemiSynchronousLambda")
            self.semi_sync_recompute_num_updates = self.specifications.get("SemiSynchronousRecomputeSteps")


class AggregationRule:
    def __init__(self, m):
        self.aggregation_rule_name = _get(m, "Name")
        self.aggregation_rule_specifications = _get(m, "RuleSpecifications", {}) or {}
        self.aggregation_rule_scaling_factor = self.aggregation_rule_specifications.get("ScalingFactor")
        self.aggregation_rule_stride_length = self.aggregation_rule_specifications.get("StrideLength", -1)

    def __str__(self):
        return (f"RuleName: {self.aggregation_rule_name}, RuleScalingFactor: "
                f"{self.aggregation_rule_scaling_factor}, RuleStrideLength: {self.aggregation_rule_stride_length}")


class GlobalModelConfig:
    def __init__(self, m):
        self.aggregation_rule = AggregationRule(_get(m, "AggregationRule"))
        self.participation_ratio = _get(m, "ParticipationRatio", 1)


_OPT_KEYS = {
    "VANILLASGD": ("VanillaSGD", {"L1Reg": "l1_reg", "L2Reg": "l2_reg"}),
    "MOMENTUMSGD": ("MomentumSGD", {"MomentumFactor": "momentum_factor"}),
    "FEDPROX": ("FedProx", {"ProximalTerm": "proximal_term"}),
    "ADAM": ("Adam", {"Beta1": "beta_1", "Beta2": "beta_2", "Epsilon": "epsilon"}),
    "ADAMW": ("AdamWeightDecay", {"WeightDecay": "weight_decay"}),
}


class OptimizerConfig:
    def __init__(self, m):
        self.optimizer_name = _get(m, "OptimizerName", "VanillaSGD")
        self.learning_rate = _get(m, "LearningRate", 0.01)
        self.optimizer_pb_kwargs = self.create_optimizer_pb_kwargs(m or {})

    def create_optimizer_pb_kwargs(self, m):
        key = self.optimizer_name.upper()
        if key not in _OPT_KEYS:
            raise RuntimeError("Not a supported optimizer.")
        name, fields = _OPT_KEYS[key]
        kw = {"name": name, "learning_rate": self.learning_rate}
        if key == "ADAMW":
            kw["weight_decay"] = 1e-4
        for yk, pk in fields.items():
            if yk in m:
                kw[pk] = m[yk]
        return kw


class LocalModelConfig:
    def __init__(self, m):
        self.batch_size = _get(m, "BatchSize", 100)
        self.local_epochs = _get(m, "LocalEpochs", 5)
        self.validation_percentage = _get(m, "ValidationPercentage", 0)
        self.optimizer_config = OptimizerConfig(_get(m, "OptimizerConfig", {}))
        self.neural_engine = _get(m, "NeuralEngine", "static")


class ConnectionConfigsBase:
    def __init__(self, m):
        self.hostname = _get(m, "Hostname")
        self.port = _get(m, "Port")


class ConnectionConfigs(ConnectionConfigsBase):
    def __init__(self, m):
        super().__init__(m)
        self.username = _get(m, "Username", "")
        self.password = _get(m, "Password", "")
        self.key_filename = _get(m, "KeyFilename", "")
        self.passphrase = _get(m, "Passphrase", "")
        self.on_login = _get(m, "OnLogin", "")


class ModelStoreConfig:
    def __init__(self, m):
        if not m:
            self.name, self.eviction_policy, self.eviction_lineage_length = "InMemory", "LineageLengthEviction", 1
            self.connection_configs = ConnectionConfigsBase({})
        else:
            self.name = m.get("Name", "InMemory")
            self.eviction_policy = m.get("EvictionPolicy", "LineageLengthEviction")
            self.eviction_lineage_length = m.get("LineageLength", 1)
            self.connection_configs = ConnectionConfigsBase(m.get("ConnectionConfigs", {}))


class GRPCServicer:
    def __init__(self, m):
        self.hostname = _get(m, "Hostname")
        self.port = _get(m, "Port")
        if not self.hostname and not self.port:
            raise RuntimeError("Malformed (hostname, port) combination. Both values need to be defined.")
        self.public_certificate_path = _get(m, "PublicCertificatePath")
        self.private_key_path = _get(m, "PrivateKeyPath")


class SSLConfigs:
    def __init__(self, m):
        self.public_certificate_file = _get(m, "PublicCertificate")
        self.private_key_file = _get(m, "PrivateKey")


class RemoteHost:
    def __init__(self, m):
        self.connection_configs = ConnectionConfigs(_get(m, "ConnectionConfigs", {}))
        self.grpc_servicer = GRPCServicer(_get(m, "GRPCServicer"))
        self.ssl_configs = SSLConfigs(m["SSLConfigs"]) if "SSLConfigs" in (m or {}) else None


class Controller(RemoteHost):
    def __init__(self, m):
        super().__init__(m)
        self.project_home = _get(m, "ProjectHome", "")


class DatasetConfigs:
    def __init__(self, m):
        self.train_dataset_path = _get(m, "TrainDatasetPath", "")
        self.validation_dataset_path = _get(m, "ValidationDatasetPath", "")
        self.test_dataset_path = _get(m, "TestDatasetPath", "")


class Learner(RemoteHost):
    def __init__(self, m):
        super().__init__(m)
        self.learner_id = _get(m, "LearnerID")
        self.project_home = _get(m, "ProjectHome", "")
        self.cuda_devices = list(_get(m, "Devices", _get(m, "CudaDevices", [])) or [])
        self.devices = self.cuda_devices
        self.dataset_configs = DatasetConfigs(_get(m, "DatasetConfigs", {}))

    def __str__(self):
        return (f"LearnerID: {self.learner_id}, GRPCServicer: {self.grpc_servicer.hostname}:"
                f"{self.grpc_servicer.port}, Devices: {self.devices}")


class Learners:
    def __init__(self, m):
        self.learners = [Learner(d) for d in (m or [])]

    def __iter__(self):
        return iter(self.learners)

    def __len__(self):
        return len(self.learners)

    def __getitem__(self, i):
        return self.learners[i]


class FederationEnvironment:
    def __init__(self, federation_environment_config_fp=None, config: dict | None = None):
        if config is None:
            with open(federation_environment_config_fp) as f:
                config = yaml.load(f.read(), Loader=yaml.SafeLoader)
        self.loaded_stream = config
        fe = config.get("FederationEnvironment")
        self.docker = DockerImage(fe.get("DockerImage"))
        self.launcher = fe.get("Launcher", "local")
        # "grpc" (the reference's: models travel through the controller) or
        # "rccl" (one process per GPU on this node, models averaged by an
        # RCCL all-reduce; the controller keeps the bookkeeping)
        self.data_plane = str(fe.get("DataPlane", "grpc")).lower()
        self.termination_signals = TerminationSignals(fe.get("TerminationSignals"))
        self.evaluation_metric = fe.get("EvaluationMetric", "accuracy")
        self.communication_protocol = CommunicationProtocol(fe.get("CommunicationProtocol"))
        self.global_model_config = GlobalModelConfig(fe.get("GlobalModelConfig"))
        self.local_model_config = LocalModelConfig(fe.get("LocalModelConfig"))
        self.model_store_config = ModelStoreConfig(fe.get("ModelStoreConfig"))
        self.controller = Controller(fe.get("Controller"))
        self.learners = Learners(fe.get("Learners"))
        self.homomorphic_encryption = None
        if "HomomorphicEncryption" in fe:
            self.homomorphic_encryption = HomomorphicEncryption(fe.get("HomomorphicEncryption"))
            assert (self.global_model_config.aggregation_rule.aggregation_rule_name or "").upper() == "PWA", \
                "Homomorphic encryption requires the PWA aggregation rule."
