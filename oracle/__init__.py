"""CPU oracle for the capsmi hot path -- TEST INFRASTRUCTURE ONLY.

Only tests/, bench.py's ``cpu_baseline`` leg and __graft_entry__.smoke() may import this package,
and only as the checker.  The product (cypher-for-apache-spark_amd/) never imports it.

Parity status: the reference (Scala 2.11 / Spark 2.2.1) cannot be built or run in this container
(no JVM, no Maven artefacts), so there is no oracle/_ref.  The restatements here
are pinned by the golden vectors transcribed from the reference's own acceptance tests
(tests/golden/*.json, with file:line of each source test) and by cross-checks between the two
independent restatements (relational numpy tables vs brute-force enumeration; C enumeration vs
closed form).
"""
