"""Test / baseline infrastructure (CPU restatements of the reference).  Never imported by the
product package ``dpgo_amd``."""
