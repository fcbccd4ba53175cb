"""Control plane over real gRPC on localhost: the controller servicer (native
engine behind it), learners with their own servicers, the controller /
learner clients.  Mirrors the reference's orchestration testing approach
(fake learners that echo the model, test/learner_notrain_noeval.py) plus a
real-compute path with the static ResNet on the CPU reference ops."""
import time

import numpy as np
import pytest

from metisfl_amd.proto import metis_pb2
from metisfl_amd.utils.proto_messages_factory import MetisProtoMessages as M
from metisfl_amd.utils.proto_messages_factory import ModelProtoMessages as MM
from metisfl_amd.utils.tensor_codec import model_from_arrays, model_to_arrays


def controller_params(protocol="SYNCHRONOUS", rule="FedAvg", batch=4, epochs=1, port=0, stride=0):
    opt = MM.construct_optimizer_config_pb(MM.construct_vanilla_sgd_optimizer_pb(0.01))
    return M.construct_controller_params_pb(
        M.construct_server_entity_pb("127.0.0.1", port),
        M.construct_global_model_specs(M.construct_aggregation_rule_pb(rule, "NumTrainingExamples", stride), 1.0),
        M.construct_communication_specs_pb(protocol, None, None),
        M.construct_model_store_config_pb("InMemory", "LineageLengthEviction", 1),
        M.construct_controller_modelhyperparams_pb(batch, epochs, opt, 0.0))


def start_controller(**kw):
    from metisfl_amd.controller.servicer import ControllerServicer
    srv = ControllerServicer(controller_params(**kw))
    port = srv.start()
    return srv, M.construct_server_entity_pb("127.0.0.1", port)


def start_learner(ctrl_entity, ops, tmp_path, idx, n_train=20, **kw):
    from metisfl_amd.learner.learner import Learner
    from metisfl_amd.learner.learner_servicer import LearnerServicer
    from metisfl_amd.models.model_dataset import ModelDatasetClassification
    rng = np.random.default_rng(idx)
    x = rng.standard_normal((n_train, 32, 32, 3)).astype(np.float32)
    y = rng.integers(0, 10, n_train)
    ds = ModelDatasetClassification(x, y)
    learner = Learner(M.construct_server_entity_pb("127.0.0.1", 0), ctrl_entity, ops, ds,
                      test_dataset=ModelDatasetClassification(x[:8], y[:8]),
                      learner_credentials_fp=str(tmp_path / f"cred{idx}"), **kw)
    srv = LearnerServicer(learner)
    srv.init_servicer()
    return learner, srv


def wait_for(pred, timeout=60.0, what=""):
    end = time.time() + timeout
    while time.time() < end:
        if pred():
            return
        time.sleep(0.05)
    raise AssertionError(f"timed out waiting for {what}")


def test_fake_learners_sync_rounds(tmp_path):
    from metisfl_amd.learner.fake import EchoModelOps
    from metisfl_amd.utils.grpc_controller_client import GRPCControllerClient
    from metisfl_amd.utils.grpc_learner_client import GRPCLearnerClient
    ctrl, ent = start_controller()
    client = GRPCControllerClient(ent)
    try:
        assert client.check_health_status().services_status["controller"]
        model = model_from_arrays(["w", "b"], [np.arange(6, dtype=np.float32).reshape(2, 3),
                                               np.ones(3, np.float32)])
        assert client.replace_community_model(1, model)
        learners = [start_learner(ent, EchoModelOps(0.05), tmp_path, i, n_train=10 * (i + 1)) for i in range(3)]
        wait_for(lambda: ctrl.engine.global_iteration() >= 3, what="3 sync rounds")
        parts = client.get_participating_learners()
        assert len(parts.learner) == 3
        md = client.get_runtime_metadata(0)
        assert len(md.metadata) >= 3 and md.json_metadata
        done = [m for m in md.metadata if m.completed_by_learner_id]
        assert len(done[0].completed_by_learner_id) == 3
        # community model = weighted average of identical echoes = the model
        fm = client.get_community_model_lineage(1).federated_models[0]
        names, arrays, _ = model_to_arrays(fm.model)
        assert names == ["w", "b"] and np.allclose(arrays[0], np.arange(6).reshape(2, 3))
        ids = [l.learner_id for l, _ in learners]
        tl = client.get_local_task_lineage(2, ids)
        assert set(tl.learner_task.keys()) == set(ids)
        ents = [l.learner_server_entity for l, _ in learners]
        ll = client.get_learner_local_model_lineage(1, ents)
        assert len(ll.learner_local_model) == 3 and len(ll.learner_local_model[0].model) == 1
        # driver -> learner health, evaluation lineage exists (fake learners evaluate to empty maps)
        lc = GRPCLearnerClient(ents[0])
        assert lc.check_health_status().services_status["server"]
        lc.shutdown()
        assert len(client.get_community_model_evaluation_lineage(0).community_evaluation) >= 1
        # rejoin with persisted credentials -> ALREADY_EXISTS path
        l0 = learners[0][0]
        assert l0.join_federation()
        for l, s in learners:
            GRPCLearnerClient(l.learner_server_entity).shutdown_learner()
        wait_for(lambda: ctrl.engine.num_learners() == 0, 20, "learners to leave")
        assert client.shutdown_controller()
        wait_for(ctrl.shutdown_request_received, 5, "controller shutdown")
    finally:
        client.shutdown()
        ctrl.stop()


def test_unauthenticated_and_invalid_requests(tmp_path):
    import grpc
    from metisfl_amd.utils.grpc_controller_client import GRPCControllerClient
    ctrl, ent = start_controller()
    client = GRPCControllerClient(ent)
    try:
        with pytest.raises(grpc.RpcError) as e:
            client.leave_federation("", "")
        assert e.value.code() == grpc.StatusCode.INVALID_ARGUMENT
        with pytest.raises(grpc.RpcError) as e:
            client.leave_federation("nobody:1", "token")
        assert e.value.code() == grpc.StatusCode.CANCELLED
        task = M.construct_completed_learning_task_pb(model_from_arrays(["w"], [np.ones(2, np.float32)]),
                                                      metis_pb2.TaskExecutionMetadata(), "")
        with pytest.raises(grpc.RpcError) as e:
            client.mark_task_completed("nobody:1", "token", task)
        assert e.value.code() in (grpc.StatusCode.NOT_FOUND, grpc.StatusCode.UNAUTHENTICATED,
                                  grpc.StatusCode.INVALID_ARGUMENT)
    finally:
        client.shutdown()
        ctrl.stop()


def test_static_resnet_learners_train_over_grpc(tmp_path):
    """Two learners really train (CPU reference ops, narrow ResNet-18) and the
    controller averages them; the community model differs from the initial one."""
    from metisfl_amd.models.model_def import StaticModelDef
    from metisfl_amd.models.model_ops import StaticModelOps
    from metisfl_amd.utils.grpc_controller_client import GRPCControllerClient
    mdef = StaticModelDef("resnet18", width_mult=0.125)
    init = StaticModelOps(mdef, device="cpu")
    names, trainable, values = init.get_model_weights()
    ctrl, ent = start_controller(batch=4, epochs=1)
    client = GRPCControllerClient(ent)
    try:
        client.replace_community_model(1, model_from_arrays(names, values, trainable))
        learners = [start_learner(ent, StaticModelOps(mdef, device="cpu"), tmp_path, i, n_train=8)
                    for i in range(2)]
        wait_for(lambda: ctrl.engine.global_iteration() >= 2, 240, "2 sync rounds with training")
        fm = client.get_community_model_lineage(1).federated_models[0]
        n2, a2, _ = model_to_arrays(fm.model)
        assert n2 == names
        diff = max(float(np.abs(a - b).max()) for a, b in zip(a2, values))
        assert diff > 0
        tl = client.get_local_task_lineage(1, [learners[0][0].learner_id])
        meta = list(tl.learner_task.values())[0].task_metadata[0]
        assert meta.completed_batches == 2 and meta.batch_size == 4
        assert meta.task_evaluation.training_evaluation[0].model_evaluation.metric_values["loss"]
        for l, s in learners:
            s.stop()
            l.shutdown()
    finally:
        client.shutdown()
        ctrl.stop()


def test_dead_learner_is_evicted_and_sync_rounds_continue(tmp_path):
    """Fault injection: a learner dies mid-federation (its server stops, it
    never reports).  The health monitor evicts it and the synchronous barrier
    completes with the survivors (the reference would wait forever)."""
    from metisfl_amd.controller.servicer import ControllerServicer
    from metisfl_amd.learner.fake import EchoModelOps
    from metisfl_amd.utils.grpc_controller_client import GRPCControllerClient
    srv = ControllerServicer(controller_params(), heartbeat_interval_s=0.2, heartbeat_threshold=2)
    port = srv.start()
    ent = M.construct_server_entity_pb("127.0.0.1", port)
    client = GRPCControllerClient(ent)
    try:
        client.replace_community_model(1, model_from_arrays(["w"], [np.ones(4, np.float32)]))
        learners = [start_learner(ent, EchoModelOps(0.05), tmp_path, i) for i in range(3)]
        wait_for(lambda: srv.engine.global_iteration() >= 2, what="2 rounds with 3 learners")
        victim, vsrv = learners[2]
        vsrv.stop()                      # crash: no LeaveFederation
        victim.shutdown()
        gi = srv.engine.global_iteration()
        wait_for(lambda: srv.engine.global_iteration() >= gi + 3, 30, "rounds after the crash")
        assert victim.learner_id in srv.monitor.evicted
        assert srv.engine.num_learners() == 2
        for l, s in learners[:2]:
            s.stop()
            l.shutdown()
    finally:
        client.shutdown()
        srv.stop()


def test_controller_restart_resumes_from_checkpoint(tmp_path):
    """the controller snapshots its engine; a new controller
    process on the same address restores it, re-dispatches the round and the
    still-running learners carry the federation on with their credentials."""
    import socket

    from metisfl_amd.controller.servicer import ControllerServicer
    from metisfl_amd.learner.fake import EchoModelOps
    from metisfl_amd.utils.grpc_controller_client import GRPCControllerClient
    from metisfl_amd.utils.grpc_learner_client import GRPCLearnerClient
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ckpt = str(tmp_path / "ckpt")
    params = controller_params(port=port)
    ctrl = ControllerServicer(params, heartbeat_interval_s=None, checkpoint_dir=ckpt)
    ctrl.start()
    ent = M.construct_server_entity_pb("127.0.0.1", port)
    client = GRPCControllerClient(ent)
    learners = []
    try:
        model = model_from_arrays(["w"], [np.arange(4, dtype=np.float32)])
        assert client.replace_community_model(1, model)
        learners = [start_learner(ent, EchoModelOps(0.05), tmp_path, i, n_train=10 * (i + 1)) for i in range(2)]
        wait_for(lambda: ctrl.engine.global_iteration() >= 3, what="rounds before the restart")
        ctrl.stop()
        gi = ctrl.engine.global_iteration()
        ctrl2 = ControllerServicer(params, heartbeat_interval_s=None, checkpoint_dir=ckpt)
        assert ctrl2.resumed and ctrl2.engine.num_learners() == 2
        assert ctrl2.engine.global_iteration() >= gi - 1
        ctrl2.start()
        ctrl = ctrl2
        wait_for(lambda: ctrl2.engine.global_iteration() >= gi + 2, what="rounds after the restart")
        md = client.get_runtime_metadata(0)
        assert len(md.metadata) >= gi + 1
    finally:
        for l, s in learners:
            try:
                GRPCLearnerClient(l.learner_server_entity).shutdown_learner()
            except Exception:
                pass
        client.shutdown()
        ctrl.stop()
