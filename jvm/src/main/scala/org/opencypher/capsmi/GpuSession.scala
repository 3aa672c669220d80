/*
 * GpuSession, records, graphs and entity tables over GpuTable: the CAPSSession / CAPSRecords /
 * CAPSGraphFactory / CAPSNodeTable analogues (spark-cypher/.../api/CAPSSession.scala:46-131,
 * impl/CAPSRecords.scala:45-143, impl/convert/rowToCypherMap.scala, impl/graph/CAPSGraphFactory.scala,
 * api/io/CAPSEntityTable.scala) for RelationalCypherSession[GpuTable].  Not compiled in this
 * repository (no JVM in the image); see INTEGRATION.md.
 */
package org.opencypher.capsmi

import com.sun.jna.Pointer
import com.sun.jna.ptr.{IntByReference, LongByReference, PointerByReference}
import org.opencypher.okapi.api.graph.{GraphName, Namespace, QualifiedGraphName}
import org.opencypher.okapi.api.io.conversion.{EntityMapping, NodeMapping, RelationshipMapping}
import org.opencypher.okapi.api.schema.Schema
import org.opencypher.okapi.api.table.CypherRecords
import org.opencypher.okapi.api.types._
import org.opencypher.okapi.api.value.CypherValue._
import org.opencypher.okapi.impl.exception.{IllegalArgumentException, UnsupportedOperationException}
import org.opencypher.okapi.impl.graph.CypherCatalog
import org.opencypher.okapi.ir.api.expr._
import org.opencypher.okapi.relational.api.graph.{RelationalCypherGraph, RelationalCypherGraphFactory, RelationalCypherSession}
import org.opencypher.okapi.relational.api.io.{NodeTable, RelationshipTable}
import org.opencypher.okapi.relational.api.table.{RelationalCypherRecords, RelationalCypherRecordsFactory}
import org.opencypher.okapi.relational.impl.table.RecordHeader

import scala.collection.immutable.TreeMap

/**
  * Order-preserving, stable string dictionary: CTString columns are int64 codes whose order is the
  * strings' order, so equality, comparisons, ORDER BY and min / max run on codes.  A code never
  * changes once issued; new strings take codes from the gap between their neighbours (the Python
  * mirror is capsmi.table.StringDictionary, tests/test_dictionary.py).
  */
final class StringDictionary {
  private val Lo = -(1L << 62)
  private val Hi = 1L << 62
  private var byString = TreeMap.empty[String, Long]
  private var byCode = Map.empty[Long, String]

  def encode(s: String): Long = synchronized {
    byString.getOrElse(s, {
      val lo = byString.until(s).lastOption.map(_._2).getOrElse(Lo)
      val hi = byString.from(s).headOption.map(_._2).getOrElse(Hi)
      val step = (hi - lo) / 2
      if (step < 1) throw UnsupportedOperationException(s"string dictionary: no code left next to '$s'")
      val code = lo + step
      byString += s -> code
      byCode += code -> s
      code
    })
  }

  def decode(code: Long): String = byCode.getOrElse(code, throw IllegalArgumentException("a dictionary code", code))
}

/** One device, one HIP stream (CAPSSession.local analogue). */
final class GpuSession(device: Int = 0) extends RelationalCypherSession[GpuTable] {
  import CapsmiLib.{I, check}

  override type Result = org.opencypher.okapi.relational.api.graph.RelationalCypherResult[GpuTable]
  override type Records = GpuRecords
  override type Graph = RelationalCypherGraph[GpuTable]

  implicit val self: GpuSession = this

  val handle: Pointer = {
    val out = new PointerByReference
    check(I.capsmi_session_create(device, out))
    out.getValue
  }

  val dictionary = new StringDictionary

  /** Graph tags -> number of dense ids, for the graphs GpuGraphFactory compacted (capsmi_graph_compact). */
  val denseIdsByGraph: scala.collection.mutable.Map[Set[Int], Long] = scala.collection.mutable.Map.empty

  override val catalog: CypherCatalog = new CypherCatalog

  private[opencypher] override val records: GpuRecordsFactory = GpuRecordsFactory()

  private[opencypher] override val graphs: GpuGraphFactory = GpuGraphFactory()

  /** Query parameters for CAPSMI_X_PARAM (ExprCompiler binds the ones a program references). */
  def setParams(values: Seq[CypherValue]): Unit = {
    val ps = new CapsmiParam().toArray(math.max(1, values.size)).asInstanceOf[Array[CapsmiParam]]
    values.zipWithIndex.foreach { case (v, i) =>
      val (items, isList) = v match {
        case CypherList(xs) => (xs, true)
        case x => (List(x), false)
      }
      val ty = items.collectFirst {
        case _: CypherFloat => Capsmi.F64
        case _: CypherInteger => Capsmi.I64
        case _: CypherBoolean => Capsmi.BOOL
        case _: CypherString => Capsmi.STR
      }.getOrElse(Capsmi.I64)
      val vals = new CapsmiValue().toArray(math.max(1, items.size)).asInstanceOf[Array[CapsmiValue]]
      items.zipWithIndex.foreach { case (x, k) =>
        x match {
          case CypherNull => vals(k).is_null = 1
          case CypherInteger(l) if ty == Capsmi.F64 => vals(k).ival = java.lang.Double.doubleToRawLongBits(l.toDouble)
          case CypherInteger(l) => vals(k).ival = l
          case CypherFloat(d) => vals(k).ival = java.lang.Double.doubleToRawLongBits(d)
          case CypherBoolean(b) => vals(k).ival = if (b) 1L else 0L
          case CypherString(s) => vals(k).ival = dictionary.encode(s)
          case other => throw UnsupportedOperationException(s"parameter value $other on the device path")
        }
        vals(k).write()
      }
      ps(i).`type` = ty; ps(i).is_list = if (isList) 1 else 0; ps(i).count = items.size
      ps(i).values = vals(0).getPointer; ps(i).write()
    }
    check(I.capsmi_session_set_params(handle, values.size, ps(0)))
  }

  /** Host columns to a device table (CAPSSession.readFrom / CAPSNodeTable ingest): Long, Int (widened),
    * Double, Boolean and String (dictionary-encoded) columns with optional nulls. */
  def table(columns: Seq[(String, CypherType, IndexedSeq[Any])]): GpuTable = {
    val n = columns.headOption.map(_._3.size).getOrElse(0)
    val descs = new ColDesc().toArray(math.max(1, columns.size)).asInstanceOf[Array[ColDesc]]
    val keep = columns.zipWithIndex.map { case ((name, ct, values), i) =>
      val ty = ct.material match {
        case CTInteger => Capsmi.I64
        case CTFloat => Capsmi.F64
        case CTBoolean => Capsmi.BOOL
        case CTString => Capsmi.STR
        case other => throw UnsupportedOperationException(s"column type $other on the device path")
      }
      val words = values.map {
        case null => 0L
        case l: Long => l
        case i: Int => i.toLong
        case d: Double => java.lang.Double.doubleToRawLongBits(d)
        case b: Boolean => if (b) 1L else 0L
        case s: String => dictionary.encode(s)
        case other => throw IllegalArgumentException(s"a value of type $ct", other)
      }.toArray
      val valid = if (values.contains(null)) Some(CapsmiLib.bytes(values.map(v => (if (v == null) 0 else 1).toByte).toArray)) else None
      val data = CapsmiLib.words(words)
      descs(i).name = name; descs(i).`type` = ty; descs(i).data = data; descs(i).valid = valid.orNull; descs(i).write()
      (data, valid)
    }
    val t = GpuTable(CapsmiLib.table(I.capsmi_table_from_host(handle, columns.size, descs(0), n, _)))
    keep.size // host buffers stay alive until the copy returned
    t
  }

  override def cypher(query: String, parameters: CypherMap, drivingTable: Option[CypherRecords]): Result =
    cypherOnGraph(graphs.empty, query, parameters, drivingTable)

  def close(): Unit = check(I.capsmi_session_destroy(handle))
}

case class GpuRecordsFactory(implicit session: GpuSession) extends RelationalCypherRecordsFactory[GpuTable] {
  override type Records = GpuRecords

  /** One row, no columns (CAPSRecordsFactory.unit: a DataFrame of one EmptyRow). */
  override def unit(): GpuRecords =
    GpuRecords(RecordHeader.empty, GpuTable(CapsmiLib.table(CapsmiLib.I.capsmi_table_from_host(session.handle, 0, new ColDesc, 1, _))))

  override def empty(initialHeader: RecordHeader = RecordHeader.empty): GpuRecords = {
    val cols = initialHeader.columns.toSeq.sorted.map { c =>
      val ct = initialHeader.exprFor(c).cypherType
      (c, if (ct.material.isInstanceOf[CTNode] || ct.material.isInstanceOf[CTRelationship]) CTInteger else ct, IndexedSeq.empty[Any])
    }
    GpuRecords(initialHeader, session.table(cols))
  }

  /** CAPSRecordsFactory.fromEntityTable: the entity table's columns are already Cypher-compatible
    * (capsmi_table_from_host widens Int / Float, capsmi_node_table verifies the id column). */
  override def fromEntityTable(entityTable: org.opencypher.okapi.relational.api.io.EntityTable[GpuTable]): GpuRecords =
    GpuRecords(entityTable.header, entityTable.table)

  override def from(header: RecordHeader, table: GpuTable, maybeDisplayNames: Option[Seq[String]]): GpuRecords = {
    val displayNames = maybeDisplayNames.orElse(Some(header.vars.map(_.withoutType).toSeq))
    GpuRecords(header, table, displayNames)
  }
}

case class GpuRecords(header: RecordHeader, table: GpuTable, override val logicalColumns: Option[Seq[String]] = None)
  (implicit session: GpuSession) extends RelationalCypherRecords[GpuTable] {

  override type Records = GpuRecords

  override def cache(): GpuRecords = copy(table = table.cache())

  override lazy val columnType: Map[String, CypherType] = table.columnType

  override def rows: Iterator[String => CypherValue] = table.rows

  override def iterator: Iterator[CypherMap] = table.rows.map(GpuRowToCypherMap(header))

  override def collect: Array[CypherMap] = iterator.toArray

  override def toString: String = if (header.isEmpty) "GpuRecords.empty" else s"GpuRecords(header: $header)"
}

/** rowToCypherMap (spark-cypher/.../impl/convert/rowToCypherMap.scala) over exported device rows. */
final case class GpuRowToCypherMap(header: RecordHeader) extends ((String => CypherValue) => CypherMap) {
  override def apply(row: String => CypherValue): CypherMap =
    CypherMap(header.returnItems.toSeq.map(r => r.name -> value(row, r)): _*)

  private def value(row: String => CypherValue, v: Var): CypherValue = v.cypherType.material match {
    case _: CTNode => node(row, v)
    case _: CTRelationship => relationship(row, v)
    case CTList(_) if !header.exprToColumn.contains(v) =>
      val elements = header.ownedBy(v).collect { case p: ListSegment => p }.toSeq.sortBy(_.index)
      CypherList(elements.map(value(row, _)).filterNot(_ == CypherNull))
    case _ => row(header.column(v))
  }

  private def properties(row: String => CypherValue, v: Var): CypherMap =
    CypherMap(header.propertiesFor(v).toSeq.map(p => p.key.name -> row(header.column(p))).filterNot(_._2 == CypherNull): _*)

  private def node(row: String => CypherValue, v: Var): CypherValue = row(header.column(v)) match {
    case CypherNull => CypherNull
    case CypherInteger(id) =>
      val labels = header.labelsFor(v).collect { case l if row(header.column(l)) == CypherBoolean(true) => l.label.name }
      GpuNode(id, labels, properties(row, v))
    case other => throw UnsupportedOperationException(s"node ID has to be a Long instead of $other")
  }

  private def relationship(row: String => CypherValue, v: Var): CypherValue = row(header.column(v)) match {
    case CypherNull => CypherNull
    case CypherInteger(id) =>
      val CypherInteger(source) = row(header.column(header.startNodeFor(v)))
      val CypherInteger(target) = row(header.column(header.endNodeFor(v)))
      val relType = header.typesFor(v).collect { case t if row(header.column(t)) == CypherBoolean(true) => t.relType.name }.head
      GpuRelationship(id, source, target, relType, properties(row, v))
    case other => throw UnsupportedOperationException(s"relationship ID has to be a Long instead of $other")
  }
}

/** CAPSNode / CAPSRelationship analogues (spark-cypher/.../api/value/CAPSEntity.scala). */
case class GpuNode(override val id: Long, override val labels: Set[String] = Set.empty,
                   override val properties: CypherMap = CypherMap.empty) extends CypherNode[Long] {
  override type I = GpuNode
  override def copy(id: Long = id, labels: Set[String] = labels, properties: CypherMap = properties): GpuNode =
    GpuNode(id, labels, properties)
}

case class GpuRelationship(override val id: Long, override val startId: Long, override val endId: Long,
                           override val relType: String, override val properties: CypherMap = CypherMap.empty)
  extends CypherRelationship[Long] {
  override type I = GpuRelationship
  override def copy(id: Long = id, source: Long = startId, target: Long = endId, relType: String = relType,
                    properties: CypherMap = properties): GpuRelationship =
    GpuRelationship(id, source, target, relType, properties).asInstanceOf[this.type]
}

/**
  * Entity tables: EntityTable.verify (okapi-relational/.../api/io/EntityTable.scala:59-65,155-164) runs
  * in the okapi constructor and again in libcapsmi (capsmi_node_table / capsmi_rel_table: Long non-null
  * id / source / target, canonical column order), which registers the table for the fused routes.
  * Build them with the companions' `create`.
  */
case class GpuNodeTable(override val mapping: NodeMapping, override val table: GpuTable)
  (implicit session: GpuSession) extends NodeTable(mapping, table) with RelationalCypherRecords[GpuTable] {
  override type Records = GpuNodeTable
  override def cache(): GpuNodeTable = copy(table = table.cache())
  override def rows: Iterator[String => CypherValue] = table.rows
  override def iterator: Iterator[CypherMap] = table.rows.map(GpuRowToCypherMap(header))
  override def collect: Array[CypherMap] = iterator.toArray

}

object GpuNodeTable {
  /** Registers the table's id / label columns with libcapsmi (the fused routes need it) and wraps
    * the registered handle; okapi's own verify runs in the NodeTable constructor. */
  def create(mapping: NodeMapping, table: GpuTable)(implicit session: GpuSession): GpuNodeTable = {
    val labels = mapping.optionalLabelMapping.values.toArray
    GpuNodeTable(mapping, GpuTable(CapsmiLib.table(
      CapsmiLib.I.capsmi_node_table(table.handle, mapping.sourceIdKey, labels.length, labels, _))))
  }
}

case class GpuRelationshipTable(override val mapping: RelationshipMapping, override val table: GpuTable)
  (implicit session: GpuSession) extends RelationshipTable(mapping, table) with RelationalCypherRecords[GpuTable] {
  override type Records = GpuRelationshipTable
  override def cache(): GpuRelationshipTable = copy(table = table.cache())
  override def rows: Iterator[String => CypherValue] = table.rows
  override def iterator: Iterator[CypherMap] = table.rows.map(GpuRowToCypherMap(header))
  override def collect: Array[CypherMap] = iterator.toArray

}

object GpuRelationshipTable {
  def create(mapping: RelationshipMapping, table: GpuTable)(implicit session: GpuSession): GpuRelationshipTable = {
    val types = mapping.relTypeOrSourceRelTypeKey.fold(_ => Array.empty[String], _._2.values.toArray)
    GpuRelationshipTable(mapping, GpuTable(CapsmiLib.table(CapsmiLib.I.capsmi_rel_table(table.handle,
      mapping.sourceIdKey, mapping.sourceStartNodeKey, mapping.sourceEndNodeKey, types.length, types, _))))
  }
}

/** CAPSGraphFactory analogue: graphs over entity tables (ScanGraph), unions and empty graphs come
  * from RelationalCypherGraphFactory unchanged. */
case class GpuGraphFactory(implicit val session: GpuSession) extends RelationalCypherGraphFactory[GpuTable] {
  def create(nodeTable: GpuNodeTable, entityTables: org.opencypher.okapi.relational.api.io.EntityTable[GpuTable]*): Graph =
    create(Set(0), None, nodeTable +: entityTables: _*)

  def create(tags: Set[Int], maybeSchema: Option[Schema],
             entityTables: org.opencypher.okapi.relational.api.io.EntityTable[GpuTable]*): Graph = {
    // dense ids for the fused kernels when the graph's ids do not fit one 2^30 window
    // (capsmi_graph_compact), as capsmi.table.Session.compact_if_sparse decides it
    val nodes = entityTables.collect { case n: GpuNodeTable => n.table.handle }.toArray
    val rels = entityTables.collect { case r: GpuRelationshipTable => r.table.handle }.toArray
    val spans = (nodes ++ rels).flatMap { h =>
      val (k, lo, hi) = (new IntByReference, new LongByReference, new LongByReference)
      CapsmiLib.check(CapsmiLib.I.capsmi_table_entity(h, k, lo, hi))
      if (k.getValue != 0 && hi.getValue > lo.getValue) Some((lo.getValue, hi.getValue)) else None
    }
    val compacted = spans.nonEmpty && spans.map(_._2).max - spans.map(_._1).min > (1L << 30)
    if (compacted) {
      val dense = new LongByReference
      CapsmiLib.check(CapsmiLib.I.capsmi_graph_compact(session.handle, nodes.length, nodes, rels.length, rels, dense))
      session.denseIdsByGraph += tags -> dense.getValue  // inspectable: which graphs run on a dense remap
    }
    val schema = maybeSchema.getOrElse(entityTables.map(_.schema).reduce(_ ++ _))
    new org.opencypher.okapi.relational.impl.graph.ScanGraph(entityTables, schema, tags)
  }
}
