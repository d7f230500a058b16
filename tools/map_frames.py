"""Map the native frames of a crash log onto libraries.

The crash and the maps come from two processes with the same command, so the
libraries the profiler preloads at start-up (librocprofiler-sdk, the system
HSA runtime) sit at the same distance from libc in both; the crash log's
pthread_kill frame fixes libc's base in the crashing process.  Libraries
loaded later (torch's own HIP runtime, hipBLASLt) can land elsewhere, so their
names here are a guess.  Usage: python tools/map_frames.py CRASH.log CLEAN.maps"""
import re
import subprocess
import sys

PTHREAD_KILL = None


def libc_symbol(name):
    out = subprocess.run(["nm", "-D", "/lib/x86_64-linux-gnu/libc.so.6"], capture_output=True, text=True).stdout
    for ln in out.splitlines():
        p = ln.split()
        if len(p) == 3 and p[2] == name + "@@GLIBC_2.34":
            return int(p[0], 16)
    raise SystemExit(f"{name} not in libc")


def main():
    log, maps_path = sys.argv[1], sys.argv[2]
    maps = []
    for ln in open(maps_path):
        p = ln.split()
        if len(p) >= 6:
            a, b = (int(x, 16) for x in p[0].split("-"))
            maps.append((a, b, p[1], int(p[2], 16), p[5]))
    clean_libc = min(m[0] - m[3] for m in maps if m[4].endswith("libc.so.6"))
    frames = [int(a, 16) for a in re.findall(r"@\s+(0x[0-9a-f]+)", open(log).read())]
    pk = [int(a, 16) for a in re.findall(r"@\s+(0x[0-9a-f]+) pthread_kill", open(log).read())]
    crash_libc = (pk[0] - libc_symbol("pthread_kill")) & ~0xFFF
    shift = crash_libc - clean_libc
    for a in frames:
        x = a - shift
        hit = [m for m in maps if m[0] <= x < m[1]]
        where = ", ".join(f"{m[4].rsplit('/', 1)[-1]} +{x - m[0] + m[3]:#x} ({m[2]})" for m in hit) or "?"
        print(f"{a:#x}  {where}")


if __name__ == "__main__":
    main()
