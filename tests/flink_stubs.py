"""Stub worker map-funcs mirroring the reference's src/test/python/test.py: echo, write-only,
drain-only, do-nothing, and a streaming echo for the latency test."""
import time


def test_example_coding(context):
    w = context.output_writer()
    for row in context.reader():
        w.write({"output": row["input"]})
    w.close()


def test_example_coding_without_encode(context):
    w = context.output_writer()
    for i in range(10):
        w.write({"output": f"output-{i}"})
    w.close()


def test_example_coding_without_decode(context):
    n = sum(1 for _ in context.reader())
    assert n >= 0


def test_example_coding_with_nothing(context):
    return None


def test_source_sink(context):
    w = context.output_writer()
    for row in context.reader():
        w.write({"output": row["input"], "t": time.time()})
    w.close()


def test_fail(context):
    raise RuntimeError("boom")


def test_types(context):
    w = context.output_writer()
    for row in context.reader():
        w.write(row)
    w.close()
