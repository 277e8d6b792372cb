"""Command line (reference: cmd/root.go, cmd/*.go, ctl/*.go).

    python -m pilosa_amd.cli server  [--data-dir D --bind H:P --cluster.hosts ... --gpu.mode auto]
    python -m pilosa_amd.cli import  -i INDEX -f FIELD [--host H] [--create-schema] [--clear] FILE...
    python -m pilosa_amd.cli export  -i INDEX -f FIELD [--host H] [-o OUT]
    python -m pilosa_amd.cli check   FRAGMENT_FILE...
    python -m pilosa_amd.cli inspect FRAGMENT_FILE
    python -m pilosa_amd.cli config  [--config FILE]        (resolved configuration as TOML)
    python -m pilosa_amd.cli generate-config                 (defaults as TOML)
"""
from __future__ import annotations

import argparse
import csv
import datetime as dt
import io
import json
import os
import signal
import sys
import threading
from typing import Dict, List, Optional

from pilosa_amd.shardwidth import SHARD_WIDTH  # noqa: E402


# ------------------------------------------------------------------ config plumbing
def _add_config_flags(p: argparse.ArgumentParser):
    from pilosa_amd.server.config import DEFAULTS

    def walk(d, prefix=""):
        for k, v in d.items():
            key = f"{prefix}{k}"
            if isinstance(v, dict):
                walk(v, key + ".")
            else:
                p.add_argument(f"--{key}", dest=f"cfg__{key}", default=None,
                               help=f"(default {v!r})")
    walk(DEFAULTS)


def resolve_config(args) -> "object":
    from pilosa_amd.server.config import Config
    cfg = Config()
    path = getattr(args, "config", None) or os.environ.get("PILOSA_CONFIG")
    if path:
        cfg.load_toml(path)
    cfg.load_env()
    for k, v in vars(args).items():
        if k.startswith("cfg__") and v is not None:
            cfg.set(k[5:], v)
    return cfg


# the configuration the last server command resolved (tests, --dry-run)
LAST_CONFIG: List[Optional[object]] = [None]


# ------------------------------------------------------------------ ctl options
# Flags of the import / export commands.  As with the reference's cobra +
# viper commands (cmd/root.go setAllConfig), a value comes from the flag, else
# the PILOSA_<NAME> environment variable, else the configuration file
# (--config / PILOSA_CONFIG, top-level keys), else the default.
#   name -> (type, default, short flag)
IMPORT_OPTIONS = {
    "host": (str, "localhost:10101", None), "index": (str, "", "-i"), "field": (str, "", "-f"),
    "create-schema": (bool, False, "-e"), "clear": (bool, False, None), "index-keys": (bool, False, None),
    "field-keys": (bool, False, None), "field-type": (str, "", None), "field-min": (int, 0, None),
    "field-max": (int, 0, None), "field-time-quantum": (str, "", None), "field-cache-type": (str, "ranked", None),
    "field-cache-size": (int, 50000, None), "buffer-size": (int, 10000000, "-b"), "sort": (bool, False, None),
}
EXPORT_OPTIONS = {"host": (str, "localhost:10101", None), "index": (str, "", "-i"), "field": (str, "", "-f"),
                  "output-file": (str, "", "-o")}
# what the last import / export command resolved (tests, --dry-run)
LAST_OPTIONS: Dict[str, dict] = {}


def _add_cmd_options(p: argparse.ArgumentParser, spec: dict):
    p.add_argument("-c", "--config", default=None)
    p.add_argument("--dry-run", action="store_true", help="stop after resolving the options")
    for name, (typ, default, short) in spec.items():
        flags = [f"--{name}"] + ([short] if short else [])
        if name == "output-file":
            flags.append("--output")
        dest = name.replace("-", "_")
        if typ is bool:
            p.add_argument(*flags, dest=dest, action="store_const", const=True, default=None,
                           help=f"(default {default})")
        else:
            p.add_argument(*flags, dest=dest, type=typ, default=None, help=f"(default {default!r})")


def _resolve_cmd_options(args, spec: dict, env=None) -> None:
    env = os.environ if env is None else env
    path = getattr(args, "config", None) or env.get("PILOSA_CONFIG")
    file = {}
    if path:
        import tomli
        with open(os.path.expanduser(path), "rb") as fh:
            file = tomli.load(fh)
    for name, (typ, default, _) in spec.items():
        dest = name.replace("-", "_")
        if getattr(args, dest, None) is not None:
            continue
        ev = env.get("PILOSA_" + name.replace("-", "_").upper())
        if ev not in (None, ""):
            val = ev.lower() in ("1", "true", "yes") if typ is bool else typ(ev)
        elif name in file:
            val = typ(file[name])
        else:
            val = default
        setattr(args, dest, val)
    if hasattr(args, "output_file"):
        args.output = args.output_file


def import_field_options(args) -> dict:
    """The field options an import creates its field with (ctl/import.go:
    keys, int range, time quantum, cache type / size)."""
    o = {"keys": bool(args.field_keys), "min": int(args.field_min), "max": int(args.field_max),
         "timeQuantum": args.field_time_quantum, "cacheType": args.field_cache_type,
         "cacheSize": int(args.field_cache_size)}
    return o


# ------------------------------------------------------------------ server
def _gossip_key(cfg):
    """The ``gossip.key`` file's bytes (validated by validate_gossip), or None."""
    path = cfg.get("gossip.key")
    if not path:
        return None
    from pilosa_amd.parallel.gossip_udp import load_key
    return load_key(str(path))


def cmd_server(args, stdout, stderr) -> int:
    from pilosa_amd.server.config import parse_duration
    from pilosa_amd.server.server import Server
    from pilosa_amd.utils import tracing
    from pilosa_amd.utils.logger import StandardLogger

    from pilosa_amd.server.config import ConfigError, validate_addrs, validate_gossip
    try:
        cfg = resolve_config(args)
        raw_adv = cfg.get("advertise")   # only an explicit advertise address overrides the listener's
        bind, adv = validate_addrs(cfg.get("bind"), raw_adv)
        validate_gossip(cfg)
    except (ConfigError, OSError) as e:
        print(e, file=stderr)
        return 1
    cfg.set("bind", bind)
    cfg.set("advertise", adv)
    LAST_CONFIG[0] = cfg
    if getattr(args, "dry_run", False):   # stop after configuration (cmd/root.go --dry-run)
        print("dry run", file=stderr)
        return 0
    log_stream = stderr
    if cfg.get("log-path"):
        log_stream = open(os.path.expanduser(cfg.get("log-path")), "a")
        # like server/setup_logger.go: send the process's stderr (native
        # library and interpreter messages too) to the log file
        try:
            os.dup2(log_stream.fileno(), 2)
        except OSError:
            pass
    logger = StandardLogger(log_stream, verbose=cfg.get("verbose"))
    if cfg.get("tracing.sampler-type") not in ("", "off", "none"):
        tracing.set_global_tracer(tracing.RecordingTracer())
    from pilosa_amd.parallel import mesh as M
    rank, world, _ = M.dist_env()
    if world > 1 and rank != 0:
        # one process per GPU (torch.distributed.run): non-front-end ranks own
        # shard subsets and execute what rank 0 broadcasts (parallel/mesh.py)
        return M.run_worker(cfg.data_dir(), gpu_mode=cfg.get("gpu.mode"), block=cfg.get("gpu.shard-block"),
                            timeout_s=cfg.duration("gpu.rccl-timeout"),
                            logger=logger)
    from pilosa_amd.utils import syswrap
    syswrap.set_max_map_count(cfg.get("max-map-count"))   # server.Command: syswrap.SetMaxMapCount
    bind = cfg.get("bind").split("://", 1)[-1]
    if bind.startswith(":"):
        bind = "0.0.0.0" + bind
    hosts = list(cfg.get("cluster.hosts")) + [h for h in cfg.get("gossip.seeds") if h not in cfg.get("cluster.hosts")]
    srv = Server(cfg.data_dir(), bind=bind, replica_n=cfg.get("cluster.replicas"), hosts=hosts,
                 coordinator=cfg.get("cluster.coordinator") or not hosts,
                 coordinator_uri=cfg.get("cluster.coordinator-uri") or (hosts[0] if hosts and
                                                                         not cfg.get("cluster.coordinator")
                                                                         else None),
                 gpu=cfg.get("gpu.mode"), workers=cfg.get("worker-pool-size"),
                 allowed_origins=list(cfg.get("handler.allowed-origins") or []),
                 advertise=adv if raw_adv else "",
                 max_writes=cfg.get("max-writes-per-request"),
                 anti_entropy_interval=cfg.duration("anti-entropy.interval"),
                 probe_interval=cfg.duration("gossip.probe-interval"),
                 probe_timeout=cfg.duration("gossip.probe-timeout"),
                 suspicion_mult=float(cfg.get("gossip.suspicion-mult")),
                 gossip_nodes=int(cfg.get("gossip.nodes")),
                 gossip_port=int(cfg.get("gossip.port") or 0),
                 gossip_key=_gossip_key(cfg),
                 to_the_dead_time=cfg.duration("gossip.to-the-dead-time"),
                 stream_timeout=cfg.duration("gossip.stream-timeout"),
                 gossip_interval=cfg.duration("gossip.push-pull-interval"),
                 long_query_time=cfg.duration("cluster.long-query-time"), stats=cfg.get("metric.service")
                 if cfg.get("metric.service") != "none" else "expvar", logger=logger,
                 cluster_disabled=cfg.get("cluster.disabled"), mesh_block=cfg.get("gpu.shard-block"),
                 translation_primary_url=cfg.get("translation.primary-url"),
                 tls_certificate=cfg.get("tls.certificate"), tls_key=cfg.get("tls.key"),
                 tls_skip_verify=cfg.get("tls.skip-verify"),
                 diagnostics_host=cfg.get("metric.diagnostics-host") if cfg.get("metric.diagnostics") else "",
                 gpu_device=int(cfg.get("gpu.devices")[0]) if cfg.get("gpu.devices") else None,
                 hbm_budget=int(cfg.get("gpu.hbm-budget")), mesh_timeout_s=cfg.duration("gpu.rccl-timeout"),
                 lazy_fragments=bool(cfg.get("gpu.lazy-fragments")),
                 native_http=bool(cfg.get("gpu.native-http")))
    srv.open()
    logger.printf("listening as %s (node %s, gpu=%s)", srv.uri.normalize(), srv.node.id,
                  "on" if srv.gpu is not None else "off")
    stop = threading.Event()
    for sig in (signal.SIGINT, signal.SIGTERM):
        try:
            signal.signal(sig, lambda *a: stop.set())
        except ValueError:
            pass
    if getattr(args, "_run_seconds", None):
        stop.wait(args._run_seconds)
    else:
        stop.wait()
    srv.close()
    return 0


# ------------------------------------------------------------------ import
def _client_uri(host: str):
    from pilosa_amd.parallel.cluster import URI
    return URI.parse(host)


def cmd_import(args, stdout, stderr) -> int:
    from pilosa_amd.parallel.cluster import Node
    from pilosa_amd.server.client import InternalClient

    _resolve_cmd_options(args, IMPORT_OPTIONS)
    LAST_OPTIONS["import"] = dict(vars(args), field_options=import_field_options(args))
    if args.dry_run:
        print("dry run", file=stderr)
        return 0

    if not args.index:
        print("index required", file=stderr)
        return 1
    if not args.field:
        print("field required", file=stderr)
        return 1
    if not args.paths:
        print("path required", file=stderr)
        return 1
    uri = _client_uri(args.host)
    c = InternalClient()
    if args.create_schema:
        c.create_index(uri, args.index, keys=args.index_keys)
        ftype = args.field_type or ("time" if args.field_time_quantum else "int" if (args.field_min or args.field_max)
                                    else "set")
        opts: Dict[str, object] = {"type": ftype}
        if ftype in ("set", "mutex"):
            opts.update({"keys": args.field_keys, "cacheType": args.field_cache_type,
                         "cacheSize": args.field_cache_size})
        elif ftype == "int":
            opts.update({"min": args.field_min, "max": args.field_max})
        elif ftype == "time":
            opts.update({"timeQuantum": args.field_time_quantum, "keys": args.field_keys})
        c.create_field(uri, args.index, args.field, opts)
    schema = c.schema(uri)
    idx = next((i for i in schema if i["name"] == args.index), None)
    if idx is None:
        print("index not found", file=stderr)
        return 1
    fld = next((f for f in idx.get("fields", []) if f["name"] == args.field), None)
    if fld is None:
        print("field not found", file=stderr)
        return 1
    is_int = fld["options"].get("type") == "int"
    is_bool = fld["options"].get("type") == "bool"
    use_col_keys = idx["options"].get("keys", False)
    use_row_keys = fld["options"].get("keys", False)
    node = Node("cli", uri)
    total = 0
    for path in args.paths:
        fh = sys.stdin if path == "-" else open(path, newline="")
        buf: List[list] = []
        for rnum, rec in enumerate(csv.reader(fh), 1):
            if not rec or rec[0] == "":
                continue
            err = _check_record(rec, rnum, is_int, is_bool, use_col_keys, use_row_keys)
            if err:
                print(err, file=stderr)
                return 1
            buf.append(rec)
            if len(buf) >= args.buffer_size:
                total += _flush(c, node, args, buf, is_int, use_col_keys, use_row_keys)
                buf = []
        total += _flush(c, node, args, buf, is_int, use_col_keys, use_row_keys)
        if fh is not sys.stdin:
            fh.close()
    print(f"imported {total} records", file=stderr)
    return 0


def _check_record(rec, rnum: int, is_int: bool, is_bool: bool, col_keys: bool, row_keys: bool) -> str:
    """The reference importer's per-record checks (ctl/import.go
    bufferBits / bufferValues): column count, numeric ids, timestamp format,
    bool rows.  Returns the error text, "" when the record is good."""
    if len(rec) < 2:
        return f"bad column count on row {rnum}: col={len(rec)}"
    if is_int:
        if not col_keys and not rec[0].isdigit():
            return f"invalid column id on row {rnum}: {rec[0]!r}"
        try:
            int(rec[1])
        except ValueError:
            return f"invalid value on row {rnum}: {rec[1]!r}"
        return ""
    if not row_keys and not rec[0].isdigit():
        return f"invalid row id on row {rnum}: {rec[0]!r}"
    if not col_keys and not rec[1].isdigit():
        return f"invalid column id on row {rnum}: {rec[1]!r}"
    if is_bool and not row_keys and int(rec[0]) not in (0, 1):
        return "bool field imports only support values 0 and 1"
    if len(rec) > 2 and rec[2]:
        try:
            dt.datetime.strptime(rec[2], "%Y-%m-%dT%H:%M")
        except ValueError:
            return f"invalid timestamp on row {rnum}: {rec[2]!r}"
    return ""


def _flush(c, node, args, buf, is_int, col_keys, row_keys) -> int:
    if not buf:
        return 0
    if is_int:
        if col_keys:
            c.import_values(node, args.index, args.field, 0, [], [int(r[1]) for r in buf],
                            col_keys=[r[0] for r in buf], clear=args.clear)
            return len(buf)
        by: Dict[int, list] = {}
        for r in buf:
            col = int(r[0])
            by.setdefault(col // SHARD_WIDTH, []).append((col, int(r[1])))
        for shard, pairs in sorted(by.items()):
            if args.sort:
                pairs.sort()
            c.import_values(node, args.index, args.field, shard, [p[0] for p in pairs], [p[1] for p in pairs],
                            clear=args.clear)
        return len(buf)
    ts = []
    for r in buf:
        if len(r) > 2 and r[2]:
            t = dt.datetime.strptime(r[2], "%Y-%m-%dT%H:%M")
            ts.append(int((t - dt.datetime(1970, 1, 1)).total_seconds() * 1e9))
        else:
            ts.append(0)
    if col_keys or row_keys:
        c.import_bits(node, args.index, args.field, 0, [] if row_keys else [int(r[0]) for r in buf],
                      [] if col_keys else [int(r[1]) for r in buf], ts if any(ts) else [], clear=args.clear,
                      row_keys=[r[0] for r in buf] if row_keys else [],
                      col_keys=[r[1] for r in buf] if col_keys else [])
        return len(buf)
    by2: Dict[int, list] = {}
    for r, t in zip(buf, ts):
        col = int(r[1])
        by2.setdefault(col // SHARD_WIDTH, []).append((int(r[0]), col, t))
    for shard, bits in sorted(by2.items()):
        if args.sort:
            bits.sort(key=lambda b: (b[0], b[1]))
        tt = [b[2] for b in bits]
        c.import_bits(node, args.index, args.field, shard, [b[0] for b in bits], [b[1] for b in bits],
                      tt if any(tt) else [], clear=args.clear)
    return len(buf)


# ------------------------------------------------------------------ export
def cmd_export(args, stdout, stderr) -> int:
    from pilosa_amd.server.client import InternalClient
    _resolve_cmd_options(args, EXPORT_OPTIONS)
    LAST_OPTIONS["export"] = dict(vars(args))
    if args.dry_run:
        print("dry run", file=stderr)
        return 0
    if not args.index:
        print("index required", file=stderr)      # pilosa.ErrIndexRequired
        return 1
    if not args.field:
        print("field required", file=stderr)      # pilosa.ErrFieldRequired
        return 1
    uri = _client_uri(args.host)
    c = InternalClient()
    maxs = c.max_shards(uri).get(args.index, 0)
    out = open(args.output, "w") if args.output else stdout
    for shard in range(maxs + 1):
        nodes = c.fragment_nodes(uri, args.index, shard)
        from pilosa_amd.parallel.cluster import URI
        target = URI.from_json(nodes[0]["uri"]) if nodes else uri
        out.write(c.export_csv(target, args.index, args.field, shard))
    if args.output:
        out.close()
    return 0


# ------------------------------------------------------------------ check / inspect
def _header_error(e: Exception) -> str:
    """The decoder's message, already in the reference's wording and prefixes
    (roaring/roaring.go UnmarshalBinary: "reading roaring header: ...")."""
    return str(e)


def cmd_check(args, stdout, stderr) -> int:
    """ctl/check.go: fragment files (no extension) are unmarshalled and
    consistency-checked; .cache and .snapshotting files are skipped with a
    note; the first file that cannot be read ends the run with its error."""
    from pilosa_amd import _roaring
    for p in args.paths:
        ext = os.path.splitext(p)[1]
        if ext == ".cache":
            print(f"{p}: ignoring cache file", file=stdout)
            continue
        if ext == ".snapshotting":
            print(f"{p}: ignoring snapshot file", file=stdout)
            continue
        if ext:
            continue
        try:
            with open(p, "rb") as fh:
                data = fh.read()
        except OSError as e:
            print(f"checking bitmap: opening file: {e}", file=stderr)
            return 1
        try:
            bm = _roaring.Bitmap.from_bytes(data)
        except Exception as e:  # noqa: BLE001
            print(f"checking bitmap: unmarshalling: {_header_error(e)}", file=stderr)
            return 1
        errs = bm.check()
        for line in (errs or "").strip().splitlines():
            print(f"{p}: {line}", file=stdout)
        print(f"{p}: ok", file=stdout)
    return 0


def cmd_inspect(args, stdout, stderr) -> int:
    from collections import Counter

    from pilosa_amd import _roaring
    if not args.path:
        print("path required", file=stderr)
        return 1
    if len(args.path) > 1:
        print("only one path allowed", file=stderr)
        return 1
    with open(args.path[0], "rb") as fh:
        data = fh.read()
    print("unmarshalling bitmap...", file=stderr)     # ctl/inspect.go
    try:
        bm = _roaring.Bitmap.from_bytes(data)
    except Exception as e:  # noqa: BLE001
        print(f"unmarshalling: {_header_error(e)}", file=stderr)
        return 1
    info = bm.container_info()
    types = Counter(t for _, t, _ in info)
    print("== Bitmap Info ==", file=stdout)
    print(f"Containers: {len(info)}", file=stdout)
    print(f"Operations: {bm.ops}", file=stdout)
    print(f"Bits: {bm.count()}", file=stdout)
    print(f"Types: {dict(types)}", file=stdout)
    print("", file=stdout)
    print("== Containers ==", file=stdout)
    print(f"{'KEY':>12} {'TYPE':>8} {'N':>8}", file=stdout)
    for k, t, n in info[: args.limit]:
        print(f"{k:>12} {t:>8} {n:>8}", file=stdout)
    return 0


def cmd_config(args, stdout, stderr) -> int:
    stdout.write(resolve_config(args).to_toml())
    return 0


def cmd_generate_config(args, stdout, stderr) -> int:
    from pilosa_amd.server.config import Config
    stdout.write(Config().to_toml())
    return 0


# ------------------------------------------------------------------ main
class _HelpFormatter(argparse.HelpFormatter):
    """Help laid out like the reference's cobra commands ("Usage:", "Flags:")."""

    def add_usage(self, usage, actions, groups, prefix=None):
        super().add_usage(usage, actions, groups, prefix="Usage: " if prefix is None else prefix)


class _Parser(argparse.ArgumentParser):
    def __init__(self, *a, **kw):
        kw.setdefault("formatter_class", _HelpFormatter)
        super().__init__(*a, **kw)
        self._optionals.title = "Flags"


def build_parser() -> argparse.ArgumentParser:
    p = _Parser(prog="pilosa", description="MI355X-native distributed bitmap index")
    sub = p.add_subparsers(dest="cmd", title="Available Commands", parser_class=_Parser)
    s = sub.add_parser("server", help="run a node")
    s.add_argument("-c", "--config", default=None)
    s.add_argument("--dry-run", action="store_true", help="stop after resolving the configuration")
    _add_config_flags(s)
    i = sub.add_parser("import", help="bulk load CSV data", usage="pilosa import [flags] PATH...")
    _add_cmd_options(i, IMPORT_OPTIONS)
    i.add_argument("paths", nargs="*")
    e = sub.add_parser("export", help="export a field as CSV", usage="pilosa export [flags]")
    _add_cmd_options(e, EXPORT_OPTIONS)
    ck = sub.add_parser("check", help="consistency check of fragment files")
    ck.add_argument("paths", nargs="+")
    ins = sub.add_parser("inspect", help="inspect a fragment file")
    ins.add_argument("path", nargs="*")
    ins.add_argument("--limit", type=int, default=100)
    cf = sub.add_parser("config", help="print the resolved configuration")
    cf.add_argument("-c", "--config", default=None)
    _add_config_flags(cf)
    sub.add_parser("generate-config", help="print the default configuration")
    return p


COMMANDS = {"server": cmd_server, "import": cmd_import, "export": cmd_export, "check": cmd_check,
            "inspect": cmd_inspect, "config": cmd_config, "generate-config": cmd_generate_config}


def main(argv=None, stdout=None, stderr=None) -> int:
    stdout = stdout or sys.stdout
    stderr = stderr or sys.stderr
    p = build_parser()
    args = p.parse_args(argv)
    if not args.cmd:
        p.print_help(stdout)
        return 0
    return COMMANDS[args.cmd](args, stdout, stderr)


if __name__ == "__main__":
    sys.exit(main())
