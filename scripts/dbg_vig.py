import sys; sys.path.insert(0, '.')
import numpy as np, torch
import cme213x
from cme213x.models.vigenere import create_cipher
from cme213x.ops.text import residue_histograms, sanitize, vigenere, match_counts
book = open('/root/reference/hw/hw3/programming/mobydick.txt', 'rb').read()
cc, key = create_cipher(book, 11, device='cpu', out_path=None)
cg, key2 = create_cipher(book, 11, device='cuda', out_path=None)
print('ciphers equal', np.array_equal(cc, cg), len(cc), len(cg))
t = torch.from_numpy(cc)
a = residue_histograms(t, 11).numpy(); b = residue_histograms(t.cuda(), 11).cpu().numpy()
print('rh equal', np.array_equal(a, b))
print(a[0]); print(b[0])
