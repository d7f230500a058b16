"""CPU: workload generators vs the reference attack semantics (backdoor.py,
model_poisoning.py) and the reference's own attack tests."""
import numpy as np
import torch

from flr.attacks import Backdoor, poison_batches_, sign_flip_


def test_backdoor_poisons_ten_of_hundred():  # reference tests/test_attacks.py:159-173
    a = Backdoor(trigger_size=3, target_class=0, poison_ratio=0.1, seed=42)
    imgs = torch.zeros(100, 1, 28, 28)
    labs = torch.arange(100) % 10
    idx = a.poison_client_(imgs, labs)
    assert a.num_poisoned == 10 and len(set(idx)) == 10
    np.random.seed(42)
    assert idx == np.random.choice(list(range(100)), size=10, replace=False).tolist()


def test_backdoor_trigger_position_and_labels():
    a = Backdoor(image_size=(32, 32))
    assert a.position == (28, 28)  # bottom_right = (h - size - 1, w - size - 1)
    imgs = torch.zeros(20, 3, 32, 32)
    labs = torch.full((20,), 7)
    idx = a.poison_client_(imgs, labs)
    for i in range(20):
        if i in idx:
            assert labs[i] == 0 and torch.all(imgs[i, :, 28:31, 28:31] == 1.0)
            assert imgs[i].sum() == 27.0
        else:
            assert labs[i] == 7 and imgs[i].sum() == 0


def test_poison_batches_step_major():
    K, B, steps = 3, 10, 2
    batches = [(torch.zeros(K, B, 3, 32, 32), torch.zeros(K, B, 16, dtype=torch.long), torch.full((K, B), 5))
               for _ in range(steps)]
    poison_batches_(batches, [1], Backdoor(poison_ratio=0.1))
    assert sum(int((b[2][1] == 0).sum()) for b in batches) == 2
    assert all(int((b[2][0] == 0).sum()) == 0 for b in batches)


def test_sign_flip():
    X = torch.randn(4, 7)
    ref = X.clone()
    sign_flip_(X, [0, 2])
    assert torch.equal(X[0], -ref[0]) and torch.equal(X[1], ref[1]) and torch.equal(X[2], -ref[2])
