"""Example jobs mirroring the reference's `flink-jpmml-examples` module."""
