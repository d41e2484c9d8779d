"""CU-masked streams (ops/streams.py, csrc/hip/runtime.hip): mask parsing on the CPU; on the GPU, the
probe kernel must only ever report CUs of the stream's mask -- eagerly and through a HIP graph replay."""
import pytest
import torch

from quantum_distributed_machine_learning_ris_channel_estimation_amd.ops import streams as S


def test_parse_and_mask_words():
    assert S.parse_cus("first:4", 256) == [0, 1, 2, 3]
    assert S.parse_cus("0-2+10,12", 256) == [0, 1, 2, 10, 12]
    assert S.parse_cus("stride:64:1", 256) == [1, 65, 129, 193]
    assert S.parse_cus("stride:8:3:2", 256) == [3, 11]
    w = S.mask_words(S.parse_cus("first:33", 256), 256)
    assert w[0] == 0xFFFFFFFF and w[1] == 1 and sum(w[2:]) == 0
    with pytest.raises(ValueError):
        S.mask_words([256], 256)


@pytest.mark.gpu
@pytest.mark.parametrize("graph", [False, True])
def test_masked_stream_confines_dispatch(cuda, graph):
    n_cu = torch.cuda.get_device_properties(cuda).multi_processor_count
    out = torch.zeros(2 * 2048, dtype=torch.int32, device=cuda)
    full = S.masked_stream(range(n_cu), cuda)
    with torch.cuda.stream(full):
        S.cu_probe_launch(out, spin=50)
    full.synchronize()
    universe = set(S.decode(out))
    assert len(universe) == n_cu
    # logical CU bits interleave the XCDs: the first 8k bits give k CUs on each of the 8 XCDs
    k = n_cu // 4
    s = S.masked_stream(range(k), cuda)
    assert S.stream_mask(s, n_cu) == list(range(k))
    out.zero_()
    if graph:
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            S.cu_probe_launch(out, spin=50)
        out.zero_()
        torch.cuda.synchronize()
        with torch.cuda.stream(s):
            g.replay()
    else:
        with torch.cuda.stream(s):
            S.cu_probe_launch(out, spin=50)
    s.synchronize()
    ids = set(S.decode(out))
    assert len(ids) == k, len(ids)
    assert ids <= universe
    per_xcd = {}
    for i in ids:
        per_xcd[i[0]] = per_xcd.get(i[0], 0) + 1
    assert len(per_xcd) == 8 and set(per_xcd.values()) == {k // 8}, per_xcd
