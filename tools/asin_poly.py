"""Coefficients of spectral.hpp's asin polynomial: asin(s) = s + s z P(z), z = s^2 <= 1/4.  The Taylor series of P
(c_k = (2k+2)! / (4^(k+1) ((k+1)!)^2 (2k+3))) to degree 44 in exact rationals, substituted z = (x + 1) / 8, converted
to the Chebyshev basis on x in [-1, 1], truncated to degree 11 (the dropped coefficients bound the error: 2^-49.4
relative to P(0) = 1/6), converted back to powers of z and rounded to double.  Prints the C initialiser."""
import math
from fractions import Fraction as F
from math import comb

N, DEG = 45, 11


def main():
    c = [F(math.factorial(2 * k + 2), 4 ** (k + 1) * math.factorial(k + 1) ** 2 * (2 * k + 3)) for k in range(N)]
    px = [F(0)] * N
    for k, ck in enumerate(c):
        for j in range(k + 1):
            px[j] += ck * comb(k, j) / F(8 ** k)
    T = [[F(1)], [F(0), F(1)]]
    for n in range(2, N):
        a = [F(0)] + [2 * v for v in T[n - 1]]
        b = T[n - 2] + [F(0)] * (len(a) - len(T[n - 2]))
        T.append([a[i] - b[i] for i in range(len(a))])
    d, rem = [F(0)] * N, px[:]
    for n in range(N - 1, -1, -1):
        d[n] = rem[n] / T[n][n]
        for i in range(n + 1):
            rem[i] -= d[n] * T[n][i]
    bound = sum(abs(float(v)) for v in d[DEG + 1:])
    print(f"// truncation bound {bound:.3e} = 2^{math.log2(bound * 6):.1f} of P(0)")
    px = [F(0)] * (DEG + 1)
    for n in range(DEG + 1):
        for i, v in enumerate(T[n]):
            if i <= DEG:
                px[i] += d[n] * v
    pz = [F(0)] * (DEG + 1)
    for j, cj in enumerate(px):
        for i in range(j + 1):
            pz[i] += cj * comb(j, i) * F(8 ** i) * (-1) ** (j - i)
    print("constexpr double kP[%d] = {%s};" % (DEG + 1, ", ".join(float(v).hex() for v in pz)))


if __name__ == "__main__":
    main()
