"""Builders for the ``metisfl`` protobuf messages.

Same class and method names as the reference's factory
(metisfl/utils/proto_messages_factory.py:9-658) so user code and the driver
read the same, implemented table-driven on top of the runtime-built message
classes.  Tensor (de)serialisation lives in utils/tensor_codec.py; the
reference's debug leftovers (writing /tmp/test.npy, decrypting right after
encrypting) are not reproduced.
"""
from __future__ import annotations

from google.protobuf.timestamp_pb2 import Timestamp

from metisfl_amd.proto import controller_pb2, learner_pb2, metis_pb2, model_pb2, service_common_pb2
from metisfl_amd.utils import tensor_codec

_SCALING = {
    "NUMCOMPLETEDBATCHES": metis_pb2.AggregationRuleSpecs.NUM_COMPLETED_BATCHES,
    "NUMPARTICIPANTS": metis_pb2.AggregationRuleSpecs.NUM_PARTICIPANTS,
    "NUMTRAININGEXAMPLES": metis_pb2.AggregationRuleSpecs.NUM_TRAINING_EXAMPLES,
}
_PROTOCOL = {
    "SYNCHRONOUS": metis_pb2.CommunicationSpecs.SYNCHRONOUS,
    "ASYNCHRONOUS": metis_pb2.CommunicationSpecs.ASYNCHRONOUS,
    "SEMI_SYNCHRONOUS": metis_pb2.CommunicationSpecs.SEMI_SYNCHRONOUS,
    "SEMISYNCHRONOUS": metis_pb2.CommunicationSpecs.SEMI_SYNCHRONOUS,
}


def _norm(s: str) -> str:
    return s.replace("_", "").upper() if s else ""


class ControllerServiceProtoMessages:
    @classmethod
    def construct_get_community_model_evaluation_lineage_request_pb(cls, num_backtracks):
        return controller_pb2.GetCommunityModelEvaluationLineageRequest(num_backtracks=num_backtracks)

    @classmethod
    def construct_get_community_model_lineage_request_pb(cls, num_backtracks):
        return controller_pb2.GetCommunityModelLineageRequest(num_backtracks=num_backtracks)

    @classmethod
    def construct_get_learner_local_model_lineage_request_pb(cls, num_backtracks, server_entities):
        return controller_pb2.GetLearnerLocalModelLineageRequest(
            num_backtracks=num_backtracks, server_entity=list(server_entities))

    @classmethod
    def construct_get_local_task_lineage_request_pb(cls, num_backtracks, learner_ids):
        return controller_pb2.GetLocalTaskLineageRequest(num_backtracks=num_backtracks,
                                                         learner_ids=list(learner_ids))

    @classmethod
    def construct_get_runtime_metadata_lineage_request_pb(cls, num_backtracks):
        return controller_pb2.GetRuntimeMetadataLineageRequest(num_backtracks=num_backtracks)

    @classmethod
    def construct_get_participating_learners_request_pb(cls):
        return controller_pb2.GetParticipatingLearnersRequest()

    @classmethod
    def construct_join_federation_request_pb(cls, server_entity_pb, local_dataset_spec_pb):
        return controller_pb2.JoinFederationRequest(server_entity=server_entity_pb,
                                                    local_dataset_spec=local_dataset_spec_pb)

    @classmethod
    def construct_leave_federation_request_pb(cls, learner_id, auth_token):
        return controller_pb2.LeaveFederationRequest(learner_id=learner_id, auth_token=auth_token)

    @classmethod
    def construct_mark_task_completed_request_pb(cls, learner_id, auth_token, completed_learning_task_pb):
        return controller_pb2.MarkTaskCompletedRequest(learner_id=learner_id, auth_token=auth_token,
                                                       task=completed_learning_task_pb)

    @classmethod
    def construct_replace_community_model_request_pb(cls, federated_model_pb):
        return controller_pb2.ReplaceCommunityModelRequest(model=federated_model_pb)


class LearnerServiceProtoMessages:
    @classmethod
    def construct_evaluate_model_request_pb(cls, model=None, batch_size=None, eval_train=None,
                                            eval_test=None, eval_valid=None, metrics_pb=None):
        E = learner_pb2.EvaluateModelRequest
        ds = [d for d, on in ((E.TRAINING, eval_train), (E.TEST, eval_test), (E.VALIDATION, eval_valid)) if on]
        return E(model=model, batch_size=batch_size or 0, evaluation_dataset=ds, metrics=metrics_pb)

    @classmethod
    def construct_evaluate_model_response_pb(cls, evaluation_pb=None):
        return learner_pb2.EvaluateModelResponse(evaluations=evaluation_pb)

    @classmethod
    def construct_run_task_request_pb(cls, federated_model_pb=None, learning_task_pb=None,
                                      hyperparameters_pb=None):
        return learner_pb2.RunTaskRequest(federated_model=federated_model_pb, task=learning_task_pb,
                                          hyperparameters=hyperparameters_pb)

    @classmethod
    def construct_run_task_response_pb(cls, ack_pb=None):
        return learner_pb2.RunTaskResponse(ack=ack_pb)


class MetisProtoMessages:
    @classmethod
    def construct_server_entity_pb(cls, hostname, port, ssl_config_pb=None):
        return metis_pb2.ServerEntity(hostname=hostname, port=int(port), ssl_config=ssl_config_pb)

    @classmethod
    def construct_ssl_config_pb(cls, enable_ssl=False, config_pb=None):
        pb = metis_pb2.SSLConfig(enable_ssl=enable_ssl)
        if isinstance(config_pb, metis_pb2.SSLConfigFiles):
            pb.ssl_config_files.CopyFrom(config_pb)
        elif isinstance(config_pb, metis_pb2.SSLConfigStream):
            pb.ssl_config_stream.CopyFrom(config_pb)
        return pb

    @classmethod
    def construct_ssl_config_files_pb(cls, public_certificate_file=None, private_key_file=None):
        return metis_pb2.SSLConfigFiles(public_certificate_file=public_certificate_file,
                                        private_key_file=private_key_file)

    @classmethod
    def construct_ssl_config_stream_pb(cls, public_certificate_stream=None, private_key_stream=None):
        return metis_pb2.SSLConfigStream(public_certificate_stream=public_certificate_stream,
                                         private_key_stream=private_key_stream)

    @classmethod
    def construct_he_scheme_config_pb(cls, enabled=False, crypto_context_file=None, public_key_file=None,
                                      private_key_file=None, empty_scheme_config_pb=None,
                                      ckks_scheme_config_pb=None):
        pb = metis_pb2.HESchemeConfig(enabled=enabled, crypto_context_file=crypto_context_file,
                                      public_key_file=public_key_file, private_key_file=private_key_file)
        if ckks_scheme_config_pb is not None:
            pb.ckks_scheme_config.CopyFrom(ckks_scheme_config_pb)
        else:
            pb.empty_scheme_config.CopyFrom(empty_scheme_config_pb or metis_pb2.EmptySchemeConfig())
        return pb

    @classmethod
    def construct_empty_scheme_config_pb(cls):
        return metis_pb2.EmptySchemeConfig()

    @classmethod
    def construct_ckks_scheme_config_pb(cls, batch_size, scaling_factor_bits):
        return metis_pb2.CKKSSchemeConfig(batch_size=batch_size, scaling_factor_bits=scaling_factor_bits)

    @classmethod
    def construct_dataset_spec_pb(cls, num_training_examples, num_validation_examples, num_test_examples,
                                  training_spec=None, validation_spec=None, test_spec=None,
                                  is_classification=False, is_regression=False):
        pb = metis_pb2.DatasetSpec(num_training_examples=int(num_training_examples),
                                   num_validation_examples=int(num_validation_examples),
                                   num_test_examples=int(num_test_examples))
        for kind, spec in (("training", training_spec), ("validation", validation_spec), ("test", test_spec)):
            if spec is None:
                continue
            if is_classification:
                getattr(pb, f"{kind}_classification_spec").CopyFrom(
                    cls.construct_classification_dataset_spec_pb(spec))
            elif is_regression:
                getattr(pb, f"{kind}_regression_spec").CopyFrom(cls.construct_regression_dataset_spec_pb(spec))
        return pb

    @classmethod
    def construct_classification_dataset_spec_pb(cls, class_distribution_specs=None):
        pb = metis_pb2.DatasetSpec.ClassificationDatasetSpec()
        for k, v in (class_distribution_specs or {}).items():
            pb.class_examples_num[int(k)] = int(v)
        return pb

    @classmethod
    def construct_regression_dataset_spec_pb(cls, regression_specs=None):
        r = regression_specs or {}
        return metis_pb2.DatasetSpec.RegressionDatasetSpec(
            min=r.get("min", 0.0), max=r.get("max", 0.0), mean=r.get("mean", 0.0),
            median=r.get("median", 0.0), mode=r.get("mode", 0.0), stddev=r.get("stddev", 0.0))

    @classmethod
    def construct_learning_task_pb(cls, num_local_updates, validation_dataset_pct, metrics=None):
        return metis_pb2.LearningTask(num_local_updates=num_local_updates,
                                      training_dataset_percentage_for_stratified_validation=validation_dataset_pct,
                                      metrics=cls.construct_evaluation_metrics_pb(metrics))

    @classmethod
    def construct_completed_learning_task_pb(cls, model_pb, task_execution_metadata_pb, aux_metadata):
        return metis_pb2.CompletedLearningTask(model=model_pb, execution_metadata=task_execution_metadata_pb,
                                               aux_metadata=aux_metadata)

    @classmethod
    def construct_task_execution_metadata_pb(cls, global_iteration, task_evaluation_pb, completed_epochs,
                                             completed_batches, batch_size, processing_ms_per_epoch,
                                             processing_ms_per_batch):
        return metis_pb2.TaskExecutionMetadata(
            global_iteration=global_iteration, task_evaluation=task_evaluation_pb,
            completed_epochs=completed_epochs, completed_batches=completed_batches,
            batch_size=batch_size, processing_ms_per_epoch=processing_ms_per_epoch,
            processing_ms_per_batch=processing_ms_per_batch)

    @classmethod
    def construct_task_evaluation_pb(cls, epoch_training_evaluations_pbs, epoch_validation_evaluations_pbs=None,
                                     epoch_test_evaluations_pbs=None):
        return metis_pb2.TaskEvaluation(training_evaluation=epoch_training_evaluations_pbs or [],
                                        validation_evaluation=epoch_validation_evaluations_pbs or [],
                                        test_evaluation=epoch_test_evaluations_pbs or [])

    @classmethod
    def construct_epoch_evaluation_pb(cls, epoch_id, model_evaluation_pb):
        return metis_pb2.EpochEvaluation(epoch_id=epoch_id, model_evaluation=model_evaluation_pb)

    @classmethod
    def construct_evaluation_metrics_pb(cls, metrics=None):
        if metrics is None:
            metrics = []
        if isinstance(metrics, str):
            metrics = [metrics]
        return metis_pb2.EvaluationMetrics(metric=list(metrics))

    @classmethod
    def construct_model_evaluation_pb(cls, metric_values=None):
        return metis_pb2.ModelEvaluation(metric_values={str(k): str(v) for k, v in (metric_values or {}).items()})

    @classmethod
    def construct_model_evaluations_pb(cls, training_evaluation_pb, validation_evaluation_pb, test_evaluation_pb):
        return metis_pb2.ModelEvaluations(training_evaluation=training_evaluation_pb,
                                          validation_evaluation=validation_evaluation_pb,
                                          test_evaluation=test_evaluation_pb)

    @classmethod
    def construct_hyperparameters_pb(cls, batch_size, optimizer_config_pb):
        return metis_pb2.Hyperparameters(batch_size=batch_size, optimizer=optimizer_config_pb)

    @classmethod
    def construct_controller_params_pb(cls, server_entity_pb, global_model_specs_pb, communication_specs_pb,
                                       model_store_config_pb, model_hyperparameters_pb):
        return metis_pb2.ControllerParams(server_entity=server_entity_pb,
                                          global_model_specs=global_model_specs_pb,
                                          communication_specs=communication_specs_pb,
                                          model_store_config=model_store_config_pb,
                                          model_hyperparams=model_hyperparameters_pb)

    @classmethod
    def construct_controller_modelhyperparams_pb(cls, batch_size, epochs, optimizer_pb, percent_validation):
        return metis_pb2.ControllerParams.ModelHyperparams(batch_size=batch_size, epochs=epochs,
                                                           optimizer=optimizer_pb,
                                                           percent_validation=percent_validation)

    @classmethod
    def construct_no_eviction_pb(cls):
        return metis_pb2.NoEviction()

    @classmethod
    def construct_lineage_length_eviction_pb(cls, lineage_length):
        return metis_pb2.LineageLengthEviction(lineage_length=lineage_length)

    @classmethod
    def construct_eviction_policy_pb(cls, policy_name, lineage_length):
        n = _norm(policy_name)
        if n == "NOEVICTION":
            return cls.construct_no_eviction_pb()
        if n == "LINEAGELENGTHEVICTION":
            return cls.construct_lineage_length_eviction_pb(lineage_length)
        raise RuntimeError(f"unsupported eviction policy {policy_name}")

    @classmethod
    def construct_model_store_specs_pb(cls, eviction_policy_pb):
        if isinstance(eviction_policy_pb, metis_pb2.NoEviction):
            return metis_pb2.ModelStoreSpecs(no_eviction=eviction_policy_pb)
        if isinstance(eviction_policy_pb, metis_pb2.LineageLengthEviction):
            return metis_pb2.ModelStoreSpecs(lineage_length_eviction=eviction_policy_pb)
        raise RuntimeError("Not a supported protobuff eviction policy.")

    @classmethod
    def construct_model_store_config_pb(cls, name, eviction_policy, lineage_length=None, store_hostname=None,
                                        store_port=None):
        specs = cls.construct_model_store_specs_pb(cls.construct_eviction_policy_pb(eviction_policy, lineage_length))
        n = _norm(name)
        if n == "INMEMORY":
            return metis_pb2.ModelStoreConfig(in_memory_store=cls.construct_in_memory_store_pb(specs))
        if n == "REDIS":
            return metis_pb2.ModelStoreConfig(
                redis_db_store=cls.construct_redis_store_pb(specs, store_hostname, store_port))
        raise RuntimeError(f"unsupported model store {name}")

    @classmethod
    def construct_in_memory_store_pb(cls, model_store_specs_pb):
        return metis_pb2.InMemoryStore(model_store_specs=model_store_specs_pb)

    @classmethod
    def construct_redis_store_pb(cls, model_store_specs_pb, hostname, port):
        return metis_pb2.RedisDBStore(model_store_specs=model_store_specs_pb,
                                      server_entity=cls.construct_server_entity_pb(hostname, port))

    @classmethod
    def construct_fed_avg_pb(cls):
        return metis_pb2.FedAvg()

    @classmethod
    def construct_fed_stride_pb(cls, stride_length):
        return metis_pb2.FedStride(stride_length=stride_length)

    @classmethod
    def construct_fed_rec_pb(cls):
        return metis_pb2.FedRec()

    @classmethod
    def construct_pwa_pb(cls, he_scheme_config_pb):
        return metis_pb2.PWA(he_scheme_config=he_scheme_config_pb)

    @classmethod
    def construct_aggregation_rule_specs_pb(cls, scaling_factor):
        sf = _SCALING.get(_norm(scaling_factor))
        if sf is None:
            raise RuntimeError("Unsupported scaling factor.")
        return metis_pb2.AggregationRuleSpecs(scaling_factor=sf)

    @classmethod
    def construct_aggregation_rule_pb(cls, rule_name, scaling_factor, stride_length=None, he_scheme_config_pb=None):
        specs = cls.construct_aggregation_rule_specs_pb(scaling_factor)
        n = _norm(rule_name)
        rule = metis_pb2.AggregationRule(aggregation_rule_specs=specs)
        if n == "FEDAVG":
            rule.fed_avg.CopyFrom(cls.construct_fed_avg_pb())
        elif n == "FEDSTRIDE":
            rule.fed_stride.CopyFrom(cls.construct_fed_stride_pb(stride_length or 0))
        elif n == "FEDREC":
            rule.fed_rec.CopyFrom(cls.construct_fed_rec_pb())
        elif n == "PWA":
            rule.pwa.CopyFrom(cls.construct_pwa_pb(he_scheme_config_pb))
        else:
            raise RuntimeError("Unsupported rule name.")
        return rule

    @classmethod
    def construct_global_model_specs(cls, aggregation_rule_pb, learners_participation_ratio):
        return metis_pb2.GlobalModelSpecs(aggregation_rule=aggregation_rule_pb,
                                          learners_participation_ratio=learners_participation_ratio)

    @classmethod
    def construct_communication_specs_pb(cls, protocol, semi_sync_lambda=None,
                                         semi_sync_recompute_num_updates=None):
        p = _PROTOCOL.get((protocol or "").upper(), metis_pb2.CommunicationSpecs.UNKNOWN)
        return metis_pb2.CommunicationSpecs(
            protocol=p, protocol_specs=metis_pb2.ProtocolSpecs(
                semi_sync_lambda=int(semi_sync_lambda or 0),
                semi_sync_recompute_num_updates=bool(semi_sync_recompute_num_updates)))


class ModelProtoMessages:
    class TensorSpecProto:
        @classmethod
        def numpy_array_to_proto_tensor_spec(cls, arr):
            return tensor_codec.numpy_to_tensor_spec(arr)

        @classmethod
        def proto_tensor_spec_to_numpy_array(cls, tensor_spec):
            return tensor_codec.tensor_spec_to_numpy(tensor_spec)

    @classmethod
    def construct_tensor_pb(cls, nparray, ciphertext=None):
        spec = tensor_codec.numpy_to_tensor_spec(nparray)
        if ciphertext is not None:
            spec.value = ciphertext
            return model_pb2.CiphertextTensor(tensor_spec=spec)
        return model_pb2.PlaintextTensor(tensor_spec=spec)

    @classmethod
    def construct_model_variable_pb(cls, name, trainable, tensor_pb):
        v = model_pb2.Model.Variable(name=name, trainable=trainable)
        if isinstance(tensor_pb, model_pb2.CiphertextTensor):
            v.ciphertext_tensor.CopyFrom(tensor_pb)
        else:
            v.plaintext_tensor.CopyFrom(tensor_pb)
        return v

    @classmethod
    def construct_model_pb_from_vars_pb(cls, variables):
        return model_pb2.Model(variables=list(variables))

    @classmethod
    def construct_model_pb_from_np(cls, weights_values, weights_names=None, weights_trainable=None,
                                   he_scheme=None):
        names = weights_names or [f"arr_{i}" for i in range(len(weights_values))]
        return tensor_codec.model_from_arrays(names, weights_values, weights_trainable, he_scheme)

    @classmethod
    def construct_federated_model_pb(cls, num_contributors, model_pb, global_iteration=0):
        return model_pb2.FederatedModel(num_contributors=num_contributors, global_iteration=global_iteration,
                                        model=model_pb)

    @classmethod
    def construct_vanilla_sgd_optimizer_pb(cls, learning_rate, l1_reg=0.0, l2_reg=0.0):
        return model_pb2.VanillaSGD(learning_rate=learning_rate, L1_reg=l1_reg, L2_reg=l2_reg)

    @classmethod
    def construct_momentum_sgd_optimizer_pb(cls, learning_rate, momentum_factor=0.0):
        return model_pb2.MomentumSGD(learning_rate=learning_rate, momentum_factor=momentum_factor)

    @classmethod
    def construct_fed_prox_optimizer_pb(cls, learning_rate, proximal_term=0.0):
        return model_pb2.FedProx(learning_rate=learning_rate, proximal_term=proximal_term)

    @classmethod
    def construct_adam_optimizer_pb(cls, learning_rate, beta_1=0.0, beta_2=0.0, epsilon=0.0):
        return model_pb2.Adam(learning_rate=learning_rate, beta_1=beta_1, beta_2=beta_2, epsilon=epsilon)

    @classmethod
    def construct_adam_optimizer_with_weight_decay_pb(cls, learning_rate, weight_decay):
        return model_pb2.AdamWeightDecay(learning_rate=learning_rate, weight_decay=weight_decay)

    _OPT_BUILDERS = {
        "VanillaSGD": "construct_vanilla_sgd_optimizer_pb",
        "MomentumSGD": "construct_momentum_sgd_optimizer_pb",
        "FedProx": "construct_fed_prox_optimizer_pb",
        "Adam": "construct_adam_optimizer_pb",
        "AdamWeightDecay": "construct_adam_optimizer_with_weight_decay_pb",
    }

    @classmethod
    def construct_optimizer_config_pb_from_kwargs(cls, optimizer_pb_kwargs):
        kw = dict(optimizer_pb_kwargs)
        name = kw.pop("name", None)
        if name not in cls._OPT_BUILDERS:
            raise RuntimeError("Optimizer kwargs refer to a non-supported optimizer.")
        return cls.construct_optimizer_config_pb(getattr(cls, cls._OPT_BUILDERS[name])(**kw))

    @classmethod
    def construct_optimizer_config_pb(cls, optimizer_pb):
        field = {model_pb2.VanillaSGD: "vanilla_sgd", model_pb2.MomentumSGD: "momentum_sgd",
                 model_pb2.FedProx: "fed_prox", model_pb2.Adam: "adam",
                 model_pb2.AdamWeightDecay: "adam_weight_decay"}.get(type(optimizer_pb))
        if field is None:
            raise RuntimeError("Optimizer proto message refers to a non-supported optimizer.")
        cfg = model_pb2.OptimizerConfig()
        getattr(cfg, field).CopyFrom(optimizer_pb)
        return cfg


class ServiceCommonProtoMessages:
    @classmethod
    def construct_ack_pb(cls, status, google_timestamp=None, message=None):
        ts = google_timestamp
        if ts is None:
            ts = Timestamp()
            ts.GetCurrentTime()
        return service_common_pb2.Ack(status=status, timestamp=ts, message=message)

    @classmethod
    def construct_get_services_health_status_request_pb(cls):
        return service_common_pb2.GetServicesHealthStatusRequest()

    @classmethod
    def construct_get_services_health_status_response_pb(cls, services_status):
        return service_common_pb2.GetServicesHealthStatusResponse(services_status=services_status)

    @classmethod
    def construct_shutdown_request_pb(cls):
        return service_common_pb2.ShutDownRequest()

    @classmethod
    def construct_shutdown_response_pb(cls, ack_pb):
        return service_common_pb2.ShutDownResponse(ack=ack_pb)
