"""PMML document model: parser, typed IR, field preparation and expression evaluation."""
