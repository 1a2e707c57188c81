"""Drop-in for the reference's ``util`` module (util.py:10-20) plus the
``cal_loss`` that its scripts import but the reference never defines
(main_cls.py:28, main_semseg.py:23).

``cal_loss`` is the label-smoothed cross entropy (eps = 0.2) of the
reference's own loss.py:4-21 (``cross_entropy``), which is what upstream
dgcnn.pytorch's util.cal_loss computes; the reference does not pin it further.
"""
import torch
import torch.nn.functional as F


def cal_loss(pred, gold, smoothing=True):
    """Cross entropy of (B, n_class) logits against int64 labels; with
    ``smoothing`` the target puts 1 - 0.2 on the true class and 0.2 / (n - 1)
    on every other (loss.py:4-21)."""
    target = gold.reshape(-1, 1)
    if not smoothing:
        return F.cross_entropy(pred, target.view(-1))
    eps, n = 0.2, pred.shape[1]
    soft = torch.full_like(pred, eps / (n - 1)).scatter_(1, target, 1.0 - eps)
    return torch.sum(-soft * F.log_softmax(pred, dim=1), dim=1).mean()


class IOStream:
    """print + append to a log file (util.py:10-20)."""

    def __init__(self, path):
        self.f = open(path, "a")

    def cprint(self, text):
        print(text)
        self.f.write(text + "\n")
        self.f.flush()

    def close(self):
        self.f.close()
