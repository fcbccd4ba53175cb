"""``python -m metisfl_amd.controller`` -- same CLI contract as the reference
(metisfl/controller/__main__.py:10-115): every argument is a hex-encoded
serialized proto; absent ones take the reference defaults ([::]:50051,
FedAvg + NumTrainingExamples, synchronous, batch 100 / 5 epochs / SGD 0.01,
in-memory store without eviction)."""
from __future__ import annotations

import argparse

from metisfl_amd.controller.controller_instance import ControllerInstance
from metisfl_amd.proto import metis_pb2
from metisfl_amd.utils.metis_logger import MetisLogger
from metisfl_amd.utils.proto_messages_factory import MetisProtoMessages as M
from metisfl_amd.utils.proto_messages_factory import ModelProtoMessages as MM


def _parse(hexstr, cls):
    if hexstr is None:
        return None
    pb = cls()
    pb.ParseFromString(bytes.fromhex(hexstr))
    return pb


def build_params(server_entity_hex=None, global_model_specs_hex=None, communication_specs_hex=None,
                 model_hyperparameters_hex=None, model_store_config_hex=None):
    se = _parse(server_entity_hex, metis_pb2.ServerEntity) or M.construct_server_entity_pb("[::]", 50051)
    gms = _parse(global_model_specs_hex, metis_pb2.GlobalModelSpecs) or M.construct_global_model_specs(
        M.construct_aggregation_rule_pb("FEDAVG", "NUMTRAININGEXAMPLES", None, None), 1)
    cs = _parse(communication_specs_hex, metis_pb2.CommunicationSpecs) or \
        M.construct_communication_specs_pb("SYNCHRONOUS", None, None)
    mh = _parse(model_hyperparameters_hex, metis_pb2.ControllerParams.ModelHyperparams) or \
        M.construct_controller_modelhyperparams_pb(
            100, 5, MM.construct_optimizer_config_pb(MM.construct_vanilla_sgd_optimizer_pb(0.01)), 0.0)
    ms = _parse(model_store_config_hex, metis_pb2.ModelStoreConfig) or \
        M.construct_model_store_config_pb("InMemory", "NoEviction")
    return M.construct_controller_params_pb(se, gms, cs, ms, mh)


def main(argv=None):
    p = argparse.ArgumentParser(prog="metisfl_amd.controller")
    p.add_argument("-e", "--controller_server_entity_protobuff_serialized_hexadecimal", default=None)
    p.add_argument("-g", "--global_model_specs_protobuff_serialized_hexadecimal", default=None)
    p.add_argument("-c", "--communication_specs_protobuff_serialized_hexadecimal", default=None)
    p.add_argument("-m", "--model_hyperparameters_protobuff_serialized_hexadecimal", default=None)
    p.add_argument("-s", "--model_store_config_protobuff_serialized_hexadecimal", default=None)
    p.add_argument("--checkpoint_dir", default=None,
                   help="snapshot the controller state here; resume from it if present")
    a = p.parse_args(argv)
    params = build_params(a.controller_server_entity_protobuff_serialized_hexadecimal,
                          a.global_model_specs_protobuff_serialized_hexadecimal,
                          a.communication_specs_protobuff_serialized_hexadecimal,
                          a.model_hyperparameters_protobuff_serialized_hexadecimal,
                          a.model_store_config_protobuff_serialized_hexadecimal)
    MetisLogger.info('Controller Parameters: """%s"""', params)
    inst = ControllerInstance()
    inst.start(params, checkpoint_dir=a.checkpoint_dir)
    inst.shutdown()


if __name__ == "__main__":
    main()
