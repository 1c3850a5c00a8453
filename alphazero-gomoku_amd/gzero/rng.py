"""Counter-based random streams shared by the HIP engine, the C oracle and the
reference harness.

The reference draws from the *global* ``random`` module
(``ai_agent.py:128-129,157,163,204,331,336,357-361``; ``bg_planner.py:240,267-269``),
which is seeded from OS entropy, so it defines no reproducible stream of its
own.  Parity therefore needs an injected stream.  A single sequential stream per
game would force the simulations of one move to run one after the other (each
rollout's draw count shifts the next one's numbers), so the stream is split
into independent sub-streams keyed by ``(seed, game_id, ply, sim)``:

* ``sim == 0``  ("main"): the opening ``choice`` (``ai_agent.py:157,163``),
  the no-children fallback ``choice`` (``ai_agent.py:204``) and the
  exploration ``random()`` / ``choice`` (``ai_agent.py:128-129``), in that order;
* ``sim == k >= 1``: every draw made while simulation ``k`` of the search runs
  (rollout ``choice`` calls, ``ai_agent.py:331,336,357-361``; planner draws
  ``bg_planner.py:240,267-269``).

Inside a sub-stream draw ``i`` is ``mix64(key + GOLDEN*(i+1))`` (SplitMix64
finaliser).  ``random()`` is the top 53 bits scaled by 2**-53 (exactly what
CPython's ``random.random`` does with its own 53 bits) and ``choice(seq)`` is
``seq[(draw * len(seq)) >> 64]``.

The same arithmetic lives in ``csrc/gz_rng.h`` (device + host) and
``oracle/gz_oracle.c``; ``tests/test_rng.py`` pins all three to the vectors in
``tests/golden/rng_vectors.json``.
"""

M64 = (1 << 64) - 1
GOLDEN = 0x9E3779B97F4A7C15
SIM_MAIN = 0


def mix64(z: int) -> int:
    z &= M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def stream_key(seed: int, game_id: int, ply: int, sim: int) -> int:
    k = mix64((seed + GOLDEN) & M64)
    k = mix64(k ^ ((game_id * GOLDEN) & M64))
    k = mix64((k + ((ply & 0xFFFFFFFF) << 32) + (sim & 0xFFFFFFFF)) & M64)
    return k


def draw(key: int, i: int) -> int:
    return mix64((key + GOLDEN * (i + 1)) & M64)


def to_unit(x: int) -> float:
    """53-bit float in [0, 1) exactly as the kernels compute it."""
    return (x >> 11) * (1.0 / 9007199254740992.0)


def below(x: int, n: int) -> int:
    """Index in [0, n) from one 64-bit draw (Lemire multiply-high)."""
    return (x * n) >> 64


class Stream:
    """One sub-stream; ``random()`` / ``choice()`` mirror the ``random`` module."""

    def __init__(self, key: int):
        self.key = key
        self.count = 0

    def next64(self) -> int:
        x = draw(self.key, self.count)
        self.count += 1
        return x

    def random(self) -> float:
        return to_unit(self.next64())

    def randbelow(self, n: int) -> int:
        return below(self.next64(), n)

    def choice(self, seq):
        if len(seq) == 0:
            raise IndexError("Cannot choose from an empty sequence")
        return seq[self.randbelow(len(seq))]


class StreamSet:
    """All sub-streams of one run; the current one is selected by ``(game, ply, sim)``.

    Counters persist per key so that returning to the main stream after a
    simulation continues where it stopped.
    """

    def __init__(self, seed: int):
        self.seed = seed
        self._streams = {}
        self.game_id = 0
        self.ply = 0
        self.sim = SIM_MAIN

    def set(self, game_id=None, ply=None, sim=None):
        if game_id is not None:
            self.game_id = game_id
        if ply is not None:
            self.ply = ply
        if sim is not None:
            self.sim = sim

    def current(self) -> Stream:
        k = (self.game_id, self.ply, self.sim)
        s = self._streams.get(k)
        if s is None:
            s = Stream(stream_key(self.seed, *k))
            self._streams[k] = s
        return s

    def count(self, game_id, ply, sim) -> int:
        s = self._streams.get((game_id, ply, sim))
        return 0 if s is None else s.count

    # random-module facade -------------------------------------------------
    def random(self) -> float:
        return self.current().random()

    def choice(self, seq):
        return self.current().choice(seq)

    def sample(self, *a, **k):  # not on the self-play path
        raise RuntimeError("random.sample is not expected on the self-play path")

    def shuffle(self, *a, **k):
        raise RuntimeError("random.shuffle is not expected on the self-play path")
