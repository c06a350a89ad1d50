"""Write the PLACEHOLDER GEAR table (splitmix64, fixed seed).

This is NOT fastcdc's table. It exists so the engine, the oracle and every
parity test run end to end while the crate's real table is unavailable in this
container (tables/README.md). Both sides read the same file, so GPU-vs-oracle
parity is exact; parity against the reference's own boundaries is unpinned
until the real table replaces this file.
"""
from pathlib import Path

MASK64 = (1 << 64) - 1


def splitmix64(state):
    while True:
        state = (state + 0x9E3779B97F4A7C15) & MASK64
        z = state
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & MASK64
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & MASK64
        yield z ^ (z >> 31)


def main():
    gen = splitmix64(0x6368756E6B657221)  # "chunker!"
    lines = ["# placeholder = true  (splitmix64 seed 0x6368756E6B657221; NOT fastcdc's GEAR)"]
    lines += [f"0x{next(gen):016x}" for _ in range(256)]
    Path(__file__).with_name("fastcdc_v2020_gear.txt").write_text("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
