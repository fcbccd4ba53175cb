"""metisfl_amd: an MI355X-native federated learning framework.

Same capabilities as MetisFL (controller / learner / driver roles, the
``metisfl`` protobuf wire format, sync / semi-sync / async protocols, FedAvg /
FedStride / FedRec / CKKS-PWA aggregation), re-designed for AMD Instinct
MI355X: learners are persistent per-GPU processes whose training step runs on
hand-written gfx950 HIP kernels, and aggregation is an RCCL collective over
xGMI.
"""
__version__ = "0.1.0"
