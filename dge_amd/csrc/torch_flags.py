"""Compiler / linker flags of the installed torch for the compiled binding (gs_torch.cpp; used by the Makefile)."""
import sys
import sysconfig

import torch.utils.cpp_extension as ce

what = sys.argv[1]
if what == "cflags":
    print(" ".join(["-I" + sysconfig.get_paths()["include"]] + ["-I" + p for p in ce.include_paths()]
                   + ["-D_GLIBCXX_USE_CXX11_ABI=%d" % int(__import__("torch")._C._GLIBCXX_USE_CXX11_ABI),
                      "-DTORCH_EXTENSION_NAME=_gs_torch"]))
elif what == "ldflags":
    libs = ce.library_paths()
    print(" ".join(["-L" + p for p in libs] + ["-Wl,-rpath," + p for p in libs]
                   + ["-lc10", "-ltorch", "-ltorch_cpu", "-ltorch_python"]))
elif what == "suffix":
    print(sysconfig.get_config_var("EXT_SUFFIX"))
