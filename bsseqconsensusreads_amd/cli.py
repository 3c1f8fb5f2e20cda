"""Command lines for the Snakemake rules this package replaces.

    python -m bsseqconsensusreads_amd.cli step5 --reference FA IN.bam OUT.bam [--fastq1 F1 --fastq2 F2]
        rules convert_Bstrain, extend, groupsort_convert, callduplex (main.snake.py:121-164), and
        with --fastq1/--fastq2 also consensusduplex_to_fq (main.snake.py:167-177)
    python -m bsseqconsensusreads_amd.cli molecular IN.bam OUT.bam [--fastq1 F1 --fastq2 F2]
        rule call_consensus_reads_molecular (main.snake.py:46-55) [+ consensus_to_fq_unfiltered]

OUT.bam may be '-' to skip the BAM when only the FASTQ pair is wanted.  Errors exit non-zero with
the message on stderr, so Snakemake aborts the rule and removes partial outputs, as it does for
the reference tools (tools/2.extend_gap.py:179-180 raises on a record without MI).

step5 on one GPU streams a coordinate-sorted input (--stream auto, the default: when the header
says SO:coordinate): bounded memory whatever the input size, decode / GPU / encode overlapped,
output identical to the whole-file path (bam.step5_stream).  Other inputs are read whole
(bam.step5); --stream true insists on streaming (an unsorted input is then an error).
step5 --gpus N on a coordinate-sorted input streams too.  --multi ranks (the default;
ranks.step5_ranks): N spawned rank processes (one per GPU) each decode, compute and encode their
own key interval of the file, and this process concatenates their fragments -- no front end.
Mates on other contigs and unmapped mates are spilled and formed in a second phase.  When a
record's owner could not read it (an insert longer than the window slack) the ranks stop and the
file runs as --multi fleet (fleet.step5_stream_multi): this process reads the BAM once
and writes the outputs in order, N spawned worker processes run the family batches it deals them
through shared memory.  Both: bounded memory, output identical to --gpus 1.  Other inputs (or a run under torch.distributed.run) take the whole-file path: one
process per GPU, every rank forms the plan, batches dealt to the ranks, rank 0 writes
(bam.consensus_sharded).  --devices maps workers / ranks to device ids (default 0..N-1).
"""
from __future__ import annotations

import argparse
import json
import os
import sys


def parse(argv):
    ap = argparse.ArgumentParser(prog="bsseqconsensusreads_amd.cli")
    sub = ap.add_subparsers(dest="cmd", required=True)
    for name in ("step5", "molecular"):
        p = sub.add_parser(name)
        if name == "step5":
            p.add_argument("--reference", "-r", required=True, help="FASTA of the alignment (tools/1 --reference)")
        p.add_argument("input")
        p.add_argument("output", help="consensus BAM, or '-' for none")
        p.add_argument("--fastq1")
        p.add_argument("--fastq2")
        p.add_argument("--read-name-prefix", default=None)
        p.add_argument("--threads", type=int, default=8)
        p.add_argument("--compression", type=int, default=6)
        p.add_argument("--device", type=int, default=0)
        p.add_argument("--gpu-bgzf", default="false", choices=("true", "false"),
                       help="deflate the output BAM's and FASTQ pair's blocks on the GPU (streaming; files ~4%% larger)")
        p.add_argument("--batch-bases", type=int, default=None, help="device batch budget in bases")
        p.add_argument("--chunk-mb", type=int, default=64, help="--stream: record MiB per chunk")
        if name == "step5":
            p.add_argument("--gpus", type=int, default=1, help="one process per GPU, family batches dealt to them")
            p.add_argument("--devices", default=None, help="comma-separated device id per rank (default 0..gpus-1)")
            p.add_argument("--multi", default="ranks", choices=["ranks", "fleet"],
                           help="--gpus N on a coordinate-sorted input: ranks = each GPU's process reads, computes "
                                "and writes its own part of the file (ranks.py; fleet when a record's owner could "
                                "not read it); fleet = one process reads and writes, the GPUs' processes compute")
            p.add_argument("--stream", default="auto", choices=["auto", "true", "false"],
                           help="bounded-memory pipelined step (bam.step5_stream; coordinate-sorted input); "
                                "false = read the whole BAM first (bam.step5); auto = stream when the header "
                                "says SO:coordinate")
        else:
            p.add_argument("--min-consensus-base-quality", type=int, default=0,
                           help="mask single-strand calls below this phred to N (main.snake.py:54 passes 0)")
            p.add_argument("--stream", default="true", choices=["true", "false"],
                           help="bounded-memory pipelined step cut between MI runs (bam.molecular_stream; the "
                                "GroupReadsByUmi order of the input); false = read the whole BAM first")
        p.add_argument("--output-per-base-tags", default="true", choices=["true", "false"],
                       help="fgbio's consensus tags (per-read and per-base statistics); off = name/SEQ/QUAL/RG/MI/RX")
    a = ap.parse_args(argv)
    if (a.fastq1 is None) != (a.fastq2 is None):
        ap.error("--fastq1 and --fastq2 go together")
    if a.output == "-" and a.fastq1 is None:
        ap.error("nothing to write: give OUT.bam or --fastq1/--fastq2")
    if a.gpu_bgzf == "true" and a.stream == "false":
        print("warning: --gpu-bgzf applies to the streaming step only; --stream false deflates on the host",
              file=sys.stderr)
    return a


def _coordinate_sorted(bam, path: str) -> bool:
    """The header's @HD SO tag says coordinate (what the streaming reader needs)."""
    for line in bam.read_bam_header(path).text.splitlines():
        if line.startswith("@HD"):
            return "\tSO:coordinate" in "\t" + line.split("\t", 1)[-1]
    return False


def _step5_fleet(a, gpus: int) -> int:
    """step5 --gpus N on a coordinate-sorted input: ranks.step5_ranks, or fleet.step5_stream_multi
    (module docstring)."""
    from . import ranks  # (fleet, with torch, only if it runs)
    devs = [int(x) for x in a.devices.split(",")] if a.devices else list(range(gpus))
    if len(devs) != gpus:
        print("--devices needs %d ids" % gpus, file=sys.stderr)
        return 2
    if a.multi == "ranks":
        try:
            info = ranks.step5_ranks(a.input, a.reference, None if a.output == "-" else a.output, devs,
                                     a.read_name_prefix, a.threads, a.compression,
                                     (a.fastq1, a.fastq2) if a.fastq1 else None,
                                     tags=a.output_per_base_tags == "true", chunk_bytes=a.chunk_mb << 20,
                                     batch_bases=a.batch_bases, gpu_bgzf=a.gpu_bgzf == "true", on_foreign="raise")
            print(json.dumps(info), file=sys.stderr)
            return 0
        except ranks.ForeignRecords as e:
            print("ranks: %s; running --multi fleet" % e, file=sys.stderr)
        except Exception as e:  # noqa: BLE001 -- the rule fails with the message
            print("%s: %s" % (type(e).__name__, e), file=sys.stderr)
            return 1
    from . import fleet
    try:
        info = fleet.step5_stream_multi(a.input, a.reference, None if a.output == "-" else a.output, devs,
                                        a.read_name_prefix, a.threads, a.compression,
                                        (a.fastq1, a.fastq2) if a.fastq1 else None,
                                        tags=a.output_per_base_tags == "true", chunk_bytes=a.chunk_mb << 20,
                                        batch_bases=a.batch_bases, gpu_bgzf=a.gpu_bgzf == "true")
    except Exception as e:  # noqa: BLE001 -- the rule fails with the message
        print("%s: %s" % (type(e).__name__, e), file=sys.stderr)
        return 1
    print(json.dumps(info), file=sys.stderr)
    return 0


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else list(argv)
    a = parse(argv)
    from . import bam, shard
    gpus = getattr(a, "gpus", 1)
    if gpus > 1 and "WORLD_SIZE" not in os.environ:
        if a.stream == "true" or (a.stream == "auto" and _coordinate_sorted(bam, a.input)):
            return _step5_fleet(a, gpus)  # this process never touches the GPU
        return shard.launch(gpus, main, (argv,))  # this process never touches the GPU
    rank, world, local = shard.env_rank()
    if world != gpus:
        print("--gpus %d but WORLD_SIZE=%d" % (gpus, world), file=sys.stderr)
        return 2
    device = a.device
    if world > 1:
        devs = [int(x) for x in a.devices.split(",")] if a.devices else list(range(world))
        if len(devs) != world:
            print("--devices needs %d ids" % world, file=sys.stderr)
            return 2
        device = devs[local]
    from .device import Engine
    out = None if a.output == "-" else a.output
    fq = (a.fastq1, a.fastq2) if a.fastq1 else None
    dist = None
    try:
        dist = shard.init("gloo") if world > 1 else None  # host gather of the batch outputs only
        eng = Engine(device)
        try:
            stream = a.cmd == "step5" and world == 1 and (
                a.stream == "true" or (a.stream == "auto" and _coordinate_sorted(bam, a.input)))
            if stream:
                info = bam.step5_stream(a.input, a.reference, out, eng, a.read_name_prefix, a.threads, a.compression,
                                        fq, tags=a.output_per_base_tags == "true", chunk_bytes=a.chunk_mb << 20,
                                        batch_bases=a.batch_bases, gpu_bgzf=a.gpu_bgzf == "true")
            elif a.cmd == "step5":
                info = bam.step5(a.input, a.reference, out, eng, a.read_name_prefix, a.threads, a.compression, fq,
                                 tags=a.output_per_base_tags == "true", batch_bases=a.batch_bases, dist=dist)
            elif a.stream == "true":
                info = bam.molecular_stream(a.input, out, eng, a.read_name_prefix, a.threads, a.compression, fq,
                                            tags=a.output_per_base_tags == "true", chunk_bytes=a.chunk_mb << 20,
                                            batch_bases=a.batch_bases, gpu_bgzf=a.gpu_bgzf == "true",
                                            min_consensus_base_quality=a.min_consensus_base_quality)
            else:
                info = bam.molecular(a.input, out, eng, a.read_name_prefix, a.threads, a.compression, fq,
                                     tags=a.output_per_base_tags == "true",
                                     min_consensus_base_quality=a.min_consensus_base_quality)
        finally:
            eng.close()
    except Exception as e:  # noqa: BLE001 -- the rule fails with the message, like the tools do
        print("%s: %s" % (type(e).__name__, e), file=sys.stderr)
        return 1
    finally:
        if dist is not None:
            dist.destroy_process_group()
    if rank == 0:
        print(json.dumps(info), file=sys.stderr)
    return 0


if __name__ == "__main__":
    sys.exit(main())
