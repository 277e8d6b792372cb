"""MI355X-native distributed bitmap index with Pilosa's data model, PQL and
HTTP API.  Host core: C++ roaring (``_roaring``), native PQL parser
(``_pql``); device core: gfx950 HIP kernels (``_hipkernels``)."""
__version__ = "v1.3.0-mi355x"
