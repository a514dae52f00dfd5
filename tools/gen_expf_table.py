#!/usr/bin/env python3
"""Generates the 2^(i/32) table used by glibc's expf (EXP2F_TABLE_BITS = 5).

glibc 2.35 sysdeps/ieee754/flt-32/e_exp2f_data.c stores
    tab[i] = asuint64(RN_double(2^(i/32))) - (i << 47),   i = 0..31
(the "- (i << 47)" pre-subtracts the exponent contribution that expf adds back
as ki << 47).  This script recomputes those words from first principles with
60-digit decimal arithmetic and prints them as C initialisers.  The result is
checked exhaustively against the system libm expf by tests/test_expf.py.
"""
import decimal
import struct


def table():
    decimal.getcontext().prec = 60
    ln2 = decimal.Decimal(2).ln()
    out = []
    for i in range(32):
        v = (decimal.Decimal(i) / 32 * ln2).exp()
        d = float(v)  # correctly rounded (via the shortest-repr-exact decimal string)
        # float(Decimal) goes through str -> correctly rounded; double check with neighbours
        bits = struct.unpack('<Q', struct.pack('<d', d))[0]
        out.append((bits - (i << 47)) & 0xFFFFFFFFFFFFFFFF)
    return out


if __name__ == '__main__':
    t = table()
    for i in range(0, 32, 2):
        print('    0x%016xULL, 0x%016xULL,' % (t[i], t[i + 1]))
