"""Driver run by tests/test_native_sanitizers.py under the ASan runtime (LD_PRELOAD) against an
``-fsanitize=address,undefined`` build of csrc/host/sexpr.c: a seeded random corpus over the
network-facing entry points (scan / to_dict / generate), deep nesting past the 512 limit,
huge and malformed canonical lengths, long tokens and non-ASCII text — every result compared
with the pure-Python codec of utils/sexpr.py.  Prints SEXPR_ASAN_OK n=<cases>."""
import importlib.util
import random
import sys

sys.path.insert(0, sys.argv[2])
spec = importlib.util.spec_from_file_location("_sexpr", sys.argv[1])
native = importlib.util.module_from_spec(spec)
spec.loader.exec_module(native)
from aiko_services_amd.utils import sexpr as S  # noqa: E402

ALPHA = list("ab01239:() \t\n'\"xT@/.-_") + ["é", "²", "漢", "\x00"]


def outcome(fn, *a):
    try:
        return ("ok", fn(*a))
    except ValueError as exc:
        return ("ValueError", str(exc))
    except RecursionError:
        return ("RecursionError", "")


def depth(text):
    d = m = 0
    for c in text:
        d += c == "("
        m = max(m, d)
        d -= c == ")" and d > 0
    return m


def rand_text(r, n):
    return "".join(r.choice(ALPHA) for _ in range(r.randint(0, n)))


def rand_expr(r, depth=0):
    k = r.random()
    if depth > 4 or k < 0.35:
        return r.choice([None, rand_text(r, 12), r.randint(-10**9, 10**9), r.random() * 1e6, True, False,
                         "12:" + rand_text(r, 4), "", "key:"])
    if k < 0.7:
        return [rand_expr(r, depth + 1) for _ in range(r.randint(0, 5))]
    if k < 0.85:
        return tuple(rand_expr(r, depth + 1) for _ in range(r.randint(0, 3)))
    return {rand_text(r, 5) or "k": rand_expr(r, depth + 1) for _ in range(r.randint(0, 3))}


def main():
    maps = open("/proc/self/maps").read()
    assert "libasan" in maps and "libubsan" in maps, "sanitizer runtimes not loaded"
    r = random.Random(1234)
    n = 0
    corpus = [rand_text(r, 80) for _ in range(6000)]
    corpus += ["(" * d + ")" * d for d in (1, 100, 511, 512, 513, 600, 5000)]
    corpus += ["(" * 700, ")" * 50, "(a (b (c" * 200]
    corpus += ["99999999999999999999999:abc", "18446744073709551616:x", "9223372036854775807:",
               "4294967296:" + "z" * 10, "00000000000000000000001:x", "3:ab", "0:", ":", "1:", "(2:ab 2:c)"]
    corpus += ["x" * 100000, "(" + " ".join(["tok"] * 50000) + ")", "'" + "é" * 5000, '"' * 3]
    for text in corpus:
        py = outcome(lambda t: S._Scanner(t).parse_list(), text)
        nat = outcome(native.scan, text)
        if nat == ("ValueError", "S-Expression nested too deeply"):
            assert depth(text) > 512, text[:80]    # the native codec's deliberate cap
            n += 1
            continue
        assert py == nat, (text[:80], py, nat)
        if py[0] == "ok":
            nd, pd = outcome(native.to_dict, py[1]), outcome(S._to_dict_py, py[1])
            if pd[0] == "RecursionError":        # the Python reference gives up first (deep trees)
                assert nd[0] in ("ok", "ValueError"), nd
            else:
                assert nd == pd, text[:80]
        n += 1
    for _ in range(4000):
        e = rand_expr(r)
        if not isinstance(e, (list, tuple, dict)):
            e = [e]
        ng, pg = outcome(native.generate, e), outcome(S._generate_py, e)
        assert ng == pg or pg[0] == "RecursionError", repr(e)[:120]
        n += 1
    deep = []
    for _ in range(2000):
        deep = [deep]
    for fn in (native.generate, native.to_dict):
        kind, _ = outcome(fn, deep)
        assert kind in ("ValueError", "RecursionError", "ok"), kind
        n += 1
    print(f"SEXPR_ASAN_OK n={n}", flush=True)


if __name__ == "__main__":
    main()
