"""CPU check of the decoder of the training forward's LeakyReLU decisions (tests/test_gpu_train.py
_hip_lrelu_masks) against an encoder written from tconv_kernel's ballot (csrc/nonode.hip: word
((t ntiles + tile) 4 + wave) 4 + q, bit l set when y > 0 at column 16 tile + 4 wave + (l >> 4), channel
4 (l & 15) + q)."""
import numpy as np
import torch

from tests.test_gpu_train import _hip_lrelu_masks


def _encode(mask):   # mask [L][T][BN][64] bool, as the kernel's ballots write it
    L, T, BN, _ = mask.shape
    ntiles = (BN + 15) // 16
    words = np.zeros((L, T, ntiles, 4, 4), dtype=np.uint64)
    for layer in range(L):
        for t in range(T):
            for col in range(BN):
                tile, wave, a = col // 16, (col % 16) // 4, col % 4
                for ch in range(64):
                    if mask[layer, t, col, ch]:
                        b, q = ch // 4, ch % 4
                        words[layer, t, tile, wave, q] |= np.uint64(1) << np.uint64(16 * a + b)
    return torch.from_numpy(words.reshape(-1).view(np.float32).copy())


def test_lrelu_mask_decoder_round_trips_the_kernel_layout():
    rng = np.random.default_rng(0)
    L, T, BN = 2, 3, 37   # a partial last tile
    mask = rng.random((L, T, BN, 64)) < 0.5
    state = torch.cat([_encode(mask), torch.full((100,), 7.0)])   # the rest of the state follows
    got = _hip_lrelu_masks(state, L, T, BN)
    for layer in range(L):
        assert np.array_equal(got[layer].numpy(), mask[layer])
