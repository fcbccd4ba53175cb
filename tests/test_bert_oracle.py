"""The BERT learner's architecture (models/bert.py, CPU reference ops) vs an
independent fp32 torch.nn BERT masked-LM (tests/torch_bert_ref.py): same
loss and the same gradient for every parameter tensor."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(__file__))


def test_bert_tiny_cpu_step_matches_torch_nn():
    from torch_bert_ref import TorchBertMLM

    from metisfl_amd.datasets import synthetic_mlm
    from metisfl_amd.models.bert import BERT_TINY, BertMLM
    from metisfl_amd.ops.optim import OptimizerSpec
    c = BERT_TINY
    rec = synthetic_mlm(8, c.seq, c.max_pred, c.vocab, seed=5, rec_stride=c.rec_stride)
    net = BertMLM(batch_size=8, device="cpu", seed=4, config=c, optimizer=OptimizerSpec("vanilla_sgd", 0.0))
    net.zero_grad_in_optimizer = False
    net._train_body(net.make_dataset(rec, shuffle=False))
    loss = float(net.stats[0]) / float(net.stats[2])
    ref = TorchBertMLM(c)
    ref.load_from_flat(net.state)
    lr = ref(torch.as_tensor(rec))
    lr.backward()
    assert abs(loss - float(lr.detach())) < 1e-3 * float(lr.detach())
    for name, gr in ref.grads_like_flat().items():
        gg = net.state.grad(name).double().reshape(gr.shape)
        gr = gr.double()
        if name == "emb.word":
            gr, gg = gr[: c.vocab], gg[: c.vocab]
        cs = float((gg * gr).sum() / (gg.norm() * gr.norm() + 1e-30))
        assert cs > 0.9995, (name, cs)
