"""symbolize_stacks.py — name the frames of a backtrace_symbols_fd dump (op_body's watchdog) made on
the GPU box: "module(+0xOFF) [0xADDR]" lines of modules built in this tree are mapped to the local
copy (the box ran this tree's build) and named with addr2line -f -C; other lines pass through.

usage: python3 tools/symbolize_stacks.py FILE [FILE ...]"""
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FRAME = re.compile(r"^(?P<mod>[^()\s]+)\((?P<sym>[^)+]*)\+?(?P<off>0x[0-9a-f]+)?\)\s*\[(?P<addr>0x[0-9a-f]+)\]")


def local(mod):
    for key in ("/repo/", "/root/repo/"):
        if key in mod:
            p = os.path.join(REPO, mod.split(key, 1)[1])
            if os.path.exists(p):
                return p
    return mod if os.path.exists(mod) else None


def name(mod, off):
    p = local(mod)
    if not p or not off:
        return None
    try:
        out = subprocess.run(["addr2line", "-f", "-C", "-e", p, off], capture_output=True, text=True, timeout=10).stdout
    except (OSError, subprocess.SubprocessError):
        return None
    fn = out.splitlines()[0] if out else "??"
    return None if fn == "??" else fn


def main():
    for path in sys.argv[1:]:
        with open(path, errors="replace") as f:
            for line in f:
                m = FRAME.match(line.strip())
                if m and not m.group("sym") and m.group("off"):
                    fn = name(m.group("mod"), m.group("off"))
                    if fn:
                        print("    %s  [%s+%s]" % (fn, os.path.basename(m.group("mod")), m.group("off")))
                        continue
                print(line.rstrip())


if __name__ == "__main__":
    main()
