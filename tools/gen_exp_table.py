#!/usr/bin/env python3
"""Generates the 2^(k/128) table of glibc's double exp (EXP_TABLE_BITS = 7).

glibc 2.35 sysdeps/ieee754/dbl-64/exp_data.c stores, for k = 0..127,
    2^(k/N) ~= H[k] * (1 + T[k])
    tab[2k]   = asuint64(T[k])                   (relative tail)
    tab[2k+1] = asuint64(H[k]) - (k << 52) / N   (H[k] = RN(2^(k/N)))
This script recomputes those words with 80-digit decimal arithmetic and
prints them as C initialisers for xrt_device.h (xrt_exp_tab).  --check
compares them with the table inside the system libm.so.6 (found by content:
it is a private symbol) -- all 256 words equal on glibc 2.35; the function
itself is checked against libm exp by tests/test_abi.py.
"""
import decimal
import struct
import sys

N = 128


def u64(x):
    return struct.unpack('<Q', struct.pack('<d', x))[0]


def table():
    decimal.getcontext().prec = 80
    out = []
    for k in range(N):
        exact = decimal.Decimal(2) ** (decimal.Decimal(k) / N)
        h = float(exact)                          # correctly rounded
        t = float(exact / decimal.Decimal(h) - 1)
        out.append(u64(t))
        out.append((u64(h) - (k << 45)) & 0xFFFFFFFFFFFFFFFF)
    return out


if __name__ == '__main__':
    t = table()
    if '--check' in sys.argv:
        data = open('/lib/x86_64-linux-gnu/libm.so.6', 'rb').read()
        blob = b''.join(struct.pack('<Q', v) for v in t)
        print('libm table found' if data.find(blob) >= 0 else 'libm table NOT found')
    else:
        for i in range(0, 2 * N, 4):
            print('        ' + ' '.join('0x%016xULL,' % v for v in t[i:i + 4]))
