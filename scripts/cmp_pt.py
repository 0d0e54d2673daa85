"""Development aid: two torch.save'd dicts of tensors bit-identical?  usage: cmp_pt.py A.pt B.pt"""
import sys

import torch

a, b = torch.load(sys.argv[1], weights_only=True), torch.load(sys.argv[2], weights_only=True)
bad = [k for k in a if not torch.equal(a[k], b[k])]
print("bit-identical" if not bad else f"DIFFER at {bad}")
sys.exit(1 if bad else 0)
