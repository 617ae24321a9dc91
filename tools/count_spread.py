"""How far apart do the shape counts drift under the reference's draw rule
(_choose_shape, tetris_env.py:183-191: weights 5 + max(counts) - count_i,
randint over CPython's MT)?  The engine's draw word holds max - count_i in a
nibble and escapes to the full counts beyond 15; this prints the
histogram of max - min over every draw of several seeded sequences.
usage: python tools/count_spread.py SEEDS DRAWS"""
import random
import sys


def run(seed, draws):
    r = random.Random(seed)
    c = [0] * 7
    hist = {}
    for _ in range(draws):
        mx = max(c)
        m = [5 + mx - x for x in c]
        v = r.randint(1, sum(m))
        s = 0
        for i, w in enumerate(m):
            s += w
            if v <= s:
                c[i] += 1
                break
        sp = max(c) - min(c)
        hist[sp] = hist.get(sp, 0) + 1
    return hist


if __name__ == "__main__":
    tot = {}
    for seed in range(int(sys.argv[1])):
        for k, v in run(seed, int(sys.argv[2])).items():
            tot[k] = tot.get(k, 0) + v
    n = sum(tot.values())
    print("spread histogram:", sorted(tot.items()))
    print("P(spread > 15) per draw = %.2e" % (sum(v for k, v in tot.items() if k > 15) / n))
