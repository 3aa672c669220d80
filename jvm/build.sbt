// The JVM side of the capsmi drop-in: a GpuTable backend for CAPS's relational planner.
// Not built in this repository (the image has no JVM); versions follow the reference's pom.xml.
name := "capsmi-caps"
organization := "org.opencypher"
scalaVersion := "2.11.12"

libraryDependencies ++= Seq(
  "org.opencypher" % "okapi-relational" % "0.1.8-SNAPSHOT",
  "net.java.dev.jna" % "jna" % "4.5.1"
)

// libcapsmi.so (cypher-for-apache-spark_amd/capsmi/libcapsmi.so, built by __graft_entry__.build())
// must be on jna.library.path at run time.
fork := true
javaOptions += s"-Djna.library.path=${baseDirectory.value / ".." / "cypher-for-apache-spark_amd" / "capsmi"}"
