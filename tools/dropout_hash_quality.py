#!/usr/bin/env python3
"""Statistical check of candidate dropout hashes over the attention index pattern (keep
fraction, keep correlation along keys and rows, 16-bit value histogram): the shipped 2-multiply
lowbias32 vs a 1-multiply round and a 24-bit-multiply mixer (round 6).  CPU only; run: python tools/dropout_hash_quality.py"""
import numpy as np
M=0xFFFFFFFF
def lowbias32(x):
    x = x & M; x ^= x >> 16; x = (x * 0x7FEB352D) & M; x ^= x >> 15; x = (x * 0x846CA68B) & M; x ^= x >> 16; return x
def one_round(x):
    x = x & M; x ^= x >> 16; x = (x * 0x7FEB352D) & M; x ^= x >> 15; return x
def mul24(x, c): return ((x & 0xFFFFFF) * c) & M   # v_mul_u32_u24 (full rate on CDNA4)
def mix24(x):   # round 6 candidate: the two 32-bit multiplies replaced by 24-bit ones
    x = x & M; x ^= x >> 16; x = mul24(x, 0x7FEB35); x ^= x >> 15; x = mul24(x, 0x846CA7); x ^= x >> 16; return x
def seedmix(seed, hi): return lowbias32(np.uint64(seed) + np.uint64((hi * 0x9E3779B9) & M))
thr = int(round(0.1*65536))
T=1024
for name,f,seed,p_ in [(n, f, sd, pp) for n, f in (("lowbias32", lowbias32), ("1-round", one_round), ("mix24", mix24))
                         for sd in (1234567, 99) for pp in (0.1, 0.5)]:
    thr = int(round(p_*65536))
    s = np.uint64(seedmix(seed, 0))
    # a [rows x T] causal-ish block of elements: element e = row*T + k, pair e>>1
    rows=512
    e = (np.arange(rows, dtype=np.uint64)[:,None]*np.uint64(T) + np.arange(T, dtype=np.uint64)[None,:]) + np.uint64(7*T*T)
    pair = e >> np.uint64(1)
    h = f((pair & np.uint64(M)) ^ s)
    bits = np.where((e & np.uint64(1)) == 1, h >> np.uint64(16), h & np.uint64(0xFFFF))
    keep = (bits >= thr).astype(np.float64)
    p = 1 - keep.mean()
    kc = keep - keep.mean()
    def corr(a,b): return float((a*b).mean()/np.sqrt((a*a).mean()*(b*b).mean()))
    lags = [corr(kc[:, :-L], kc[:, L:]) for L in (1,2,3,4,8,16,64)]
    rowc = [corr(kc[:-L], kc[L:]) for L in (1,2,4)]
    # chi-square of 16-bit value histogram in 256 bins
    hist = np.bincount((bits >> np.uint64(8)).astype(np.int64).ravel(), minlength=256)
    exp = bits.size/256; chi = float(((hist-exp)**2/exp).sum())
    print(f"{name} seed {seed} p {p_}: drop frac {p:.5f} (target {thr/65536:.5f}), key-lag corr {[round(x,4) for x in lags]}, row-lag corr {[round(x,4) for x in rowc]}, chi2(255 dof) {chi:.0f}")
