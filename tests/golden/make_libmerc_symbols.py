"""The function names the reference's public header declares
(/root/reference/src/libmerc/libmerc.h, every `extern "C"
LIBMERC_DLL_EXPORTED` declaration), one per line, into
tests/golden/libmerc_h_symbols.txt.  Run in the dev container; the list is
data (names only), checked by tests/test_abi.py against the exports of
libmercury_amd.so and by the link test tests/c/libmerc_link.c."""
import os
import re

HERE = os.path.dirname(os.path.abspath(__file__))
HDR = "/root/reference/src/libmerc/libmerc.h"


def main():
    src = open(HDR).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    src = re.sub(r"//[^\n]*", "", src)
    names = []
    src = re.sub(r"#define LIBMERC_DLL_EXPORTED[^\n]*", "", src)
    for m in re.finditer(r"LIBMERC_DLL_EXPORTED\s*(?:#endif)?\s*([^;{]*?)\b(\w+)\s*\(", src):
        if m.group(2) not in names:
            names.append(m.group(2))
    with open(os.path.join(HERE, "libmerc_h_symbols.txt"), "w") as f:
        f.write("\n".join(names) + "\n")
    print(len(names), names)


if __name__ == "__main__":
    main()
