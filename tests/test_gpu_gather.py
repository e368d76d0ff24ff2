"""GPU: the multi-GPU NAL gather's device packing (h264mi_nal_pack / h264mi_nal_unpack, csrc/gather.inc):
a group's staged access units leave a rank as one contiguous message (unit u at the sum of the sizes before
it) and rank 0 scatters each received message back into slots. Ragged sizes with empty units and every
byte alignment of the packed offsets, against numpy."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('n,slot', [(1, 64), (37, 4096), (128, 1 << 16)])
def test_pack_unpack_round_trip(gpu_lib, n, slot):
    import torch
    rng = np.random.default_rng(n)
    sizes = rng.integers(0, slot + 1, n).astype(np.int32)
    sizes[rng.random(n) < 0.2] = 0
    if n > 1:
        sizes[1] = slot  # a full slot
    src = torch.from_numpy(rng.integers(0, 256, n * slot, dtype=np.uint8)).cuda()
    sz = torch.from_numpy(sizes).cuda()
    tot = int(sizes.sum())
    packed = torch.zeros(max(tot, 1) + 64, dtype=torch.uint8, device='cuda')
    st = torch.cuda.current_stream().cuda_stream
    assert gpu_lib.h264mi_nal_pack(packed.data_ptr(), src.data_ptr(), slot, sz.data_ptr(), n, st) == 0
    host = src.cpu().numpy()
    want = np.concatenate([host[u * slot:u * slot + int(b)] for u, b in enumerate(sizes)] + [np.zeros(0, np.uint8)])
    got = packed.cpu().numpy()
    assert np.array_equal(got[:tot], want) and not got[tot:].any()
    back = torch.zeros(n * slot, dtype=torch.uint8, device='cuda')
    assert gpu_lib.h264mi_nal_unpack(back.data_ptr(), packed.data_ptr(), slot, sz.data_ptr(), n, st) == 0
    b = back.cpu().numpy()
    for u, k in enumerate(sizes):
        assert np.array_equal(b[u * slot:u * slot + k], host[u * slot:u * slot + k]) and not b[u * slot + k:(u + 1) * slot].any()
    assert gpu_lib.h264mi_nal_pack(packed.data_ptr(), src.data_ptr(), slot, sz.data_ptr(), 0, st) == -1
