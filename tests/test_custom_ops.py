"""The torch.library surface (north_star: the hot path behind custom ops).

``sesa::{mdx23c,bsr,scnet,htdemucs}_forward``, ``sesa::chunk_gather(_into)``,
``sesa::chunk_gather_constant_into``, ``sesa::ola_accumulate`` / ``ola_counter`` / ``ola_finalize``,
``sesa::stft`` / ``istft``: registered with schemas and fake (meta) implementations, so shape
propagation works without a device (CPU tests); on the GPU ``torch.library.opcheck`` validates
schema / fake-tensor agreement against the real HIP kernels, and the nn.Module faces' forwards go
through the ops.
"""
import os
import re

import numpy as np
import pytest
import torch

from conftest import CONFIGS

OPS = ["mdx23c_forward", "bsr_forward", "scnet_forward", "htdemucs_forward", "chunk_gather", "chunk_gather_into",
       "chunk_gather_constant_into", "ola_accumulate", "ola_counter", "ola_finalize", "stft", "istft"]


def test_ops_registered_with_schemas():
    from sesa import ops  # noqa: F401
    for name in OPS:
        op = getattr(torch.ops.sesa, name)
        assert op.default._schema.name == f"sesa::{name}"
    sch = str(torch.ops.sesa.ola_accumulate.default._schema)
    assert re.search(r"Tensor\(a\d*!\) result", sch) and re.search(r"Tensor\(a\d*!\) counter", sch)  # mutations
    assert re.search(r"Tensor\(a\d*!\) workspace", str(torch.ops.sesa.bsr_forward.default._schema))


def test_fake_shapes_without_device():
    from torch._subclasses.fake_tensor import FakeTensorMode
    from sesa import ops  # noqa: F401
    with FakeTensorMode():
        x = torch.empty(3, 2, 4410)
        ws = torch.empty(64, dtype=torch.uint8)
        for net, shape in (("mdx23c", [3, 1, 2, 4410]), ("bsr", [3, 1, 2, 4410]), ("scnet", [3, 4, 2, 4410]),
                           ("htdemucs", [3, 4, 2, 4410])):
            assert getattr(torch.ops.sesa, f"{net}_forward")(0, x, ws, shape).shape == tuple(shape)
        assert torch.ops.sesa.chunk_gather(torch.empty(2, 9000), 100, [0, 500, 1000], 256).shape == (3, 2, 256)
        assert torch.ops.sesa.ola_finalize(torch.empty(4, 1200), torch.empty(1, 1200), 100).shape == (4, 1000)
        assert torch.ops.sesa.stft(torch.empty(2, 2, 8192), 1024, 256, 512).shape == (2, 2, 2, 512, 33)


def test_no_cpu_fallback():
    from sesa import ops
    from sesa._native import SesaError
    with pytest.raises((SesaError, RuntimeError)):
        ops.chunk_gather(torch.zeros(2, 100), 0, [0], 50)


@pytest.mark.gpu
def test_opcheck_chunker_and_ola():
    from sesa import ops  # noqa: F401
    dev = "cuda:0"
    rng = np.random.default_rng(0)
    mix = torch.tensor(rng.standard_normal((2, 20000)), dtype=torch.float32, device=dev)
    utils = ("test_schema", "test_faketensor")
    torch.library.opcheck(torch.ops.sesa.chunk_gather.default, (mix, 300, [0, 4000, 9000], 4096), test_utils=utils)
    out = torch.empty(3, 2, 4096, device=dev)
    torch.library.opcheck(torch.ops.sesa.chunk_gather_into.default, (mix, 300, [0, 4000, 9000], 4096, out),
                          test_utils=utils)
    y = torch.tensor(rng.standard_normal((3, 2, 4096)), dtype=torch.float32, device=dev)
    win = torch.ones(4096, device=dev)
    res = torch.zeros(2, 20600, device=dev)
    cnt = torch.zeros(1, 20600, device=dev)
    torch.library.opcheck(torch.ops.sesa.ola_accumulate.default, (y, [0, 4000, 9000], [4096, 4096, 4096], win, res, cnt),
                          test_utils=utils)
    torch.library.opcheck(torch.ops.sesa.ola_finalize.default, (res, cnt + 1.0, 300), test_utils=utils)


@pytest.mark.gpu
def test_module_forward_goes_through_op():
    """The nn.Module face dispatches sesa::mdx23c_forward (a profiler-visible op), and the op's result
    equals the module's."""
    from sesa.utils import get_model_from_config
    from sesa.weights import synth_state_dict
    model, cfg = get_model_from_config("mdx23c", os.path.join(CONFIGS, "config_mdx23c_small.yaml"))
    model.load_state_dict(synth_state_dict(model, affine="random"))
    model = model.to("cuda:0")
    x = torch.tensor(np.random.default_rng(1).standard_normal((2, 2, cfg.audio.chunk_size)) * 0.1,
                     dtype=torch.float32, device="cuda:0")
    with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU]) as prof:
        y = model(x)
    assert any(e.name == "sesa::mdx23c_forward" for e in prof.events())
    h = model._handle(x.device, x.shape[-1])
    ws = model.workspace(x.device, h, x.shape[0])
    out_shape = list(model._out_shape(x.shape[0], x.shape[1], x.shape[2]))
    torch.library.opcheck(torch.ops.sesa.mdx23c_forward.default, (h.value, x, ws, out_shape),
                          test_utils=("test_schema", "test_faketensor"))
    z = torch.ops.sesa.mdx23c_forward(h.value, x, ws, out_shape)
    assert torch.equal(model._post(z), y)
