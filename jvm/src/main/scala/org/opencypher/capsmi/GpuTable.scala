/*
 * GpuTable: Table[GpuTable] over libcapsmi device tables -- the drop-in for DataFrameTable
 * (spark-cypher/src/main/scala/org/opencypher/spark/impl/table/SparkTable.scala:47-257) behind the
 * plug-in trait okapi-relational/.../api/table/Table.scala:43-176.
 *
 * Every member is one C call; operators are lazy in libcapsmi (a plan node per call, like a
 * DataFrame), and the first action (size, rows, export) materialises the plan, routing the Expand /
 * ExpandInto / var-length shapes RelationalPlanner emits to the fused kernels
 * (cypher-for-apache-spark_amd/csrc/plan.hip).  Not compiled in this repository (no JVM in the
 * image); the Python mirror `capsmi.table.GpuTable` runs the same calls under tests/.
 */
package org.opencypher.capsmi

import java.lang.ref.Cleaner

import com.sun.jna.Pointer
import com.sun.jna.ptr.{IntByReference, LongByReference}
import org.opencypher.okapi.api.types._
import org.opencypher.okapi.api.value.CypherValue
import org.opencypher.okapi.api.value.CypherValue.{CypherList, CypherMap, CypherValue}
import org.opencypher.okapi.impl.exception.{IllegalArgumentException, NotImplementedException}
import org.opencypher.okapi.ir.api.expr._
import org.opencypher.okapi.relational.api.table.Table
import org.opencypher.okapi.relational.impl.planning._
import org.opencypher.okapi.relational.impl.table.RecordHeader

import scala.collection.mutable

object GpuTable {
  private[capsmi] val cleaner: Cleaner = Cleaner.create()

  /** Wraps an owned handle; the handle is released when the JVM object is collected. */
  def apply(handle: Pointer)(implicit session: GpuSession): GpuTable = new GpuTable(handle)

  private def joinCode(jt: JoinType): Int = jt match {
    case InnerJoin => Capsmi.JOIN_INNER
    case LeftOuterJoin => Capsmi.JOIN_LEFT_OUTER
    case RightOuterJoin => Capsmi.JOIN_RIGHT_OUTER
    case FullOuterJoin => Capsmi.JOIN_FULL_OUTER
    case CrossJoin => Capsmi.JOIN_CROSS
  }

  def cypherType(physical: Int, nullable: Boolean): CypherType = {
    val t = physical match {
      case Capsmi.I64 => CTInteger
      case Capsmi.BOOL => CTBoolean
      case Capsmi.F64 => CTFloat
      case Capsmi.STR => CTString
      case l if l >= Capsmi.LIST && l <= Capsmi.LIST + Capsmi.STR => CTList(cypherType(l - Capsmi.LIST, nullable = false))
      case other => throw IllegalArgumentException("a capsmi column type", other)
    }
    if (nullable) t.nullable else t
  }

  /** Rows exported per host round trip (rows() streams a table of any size in chunks of this). */
  private val ExportChunk = 1 << 20

  private def decode(ty: Int, w: Long)(implicit session: GpuSession): CypherValue = ty match {
    case Capsmi.I64 => CypherValue(w)
    case Capsmi.F64 => CypherValue(java.lang.Double.longBitsToDouble(w))
    case Capsmi.BOOL => CypherValue(w != 0)
    case Capsmi.STR => CypherValue(session.dictionary.decode(w))
  }
}

final class GpuTable private (val handle: Pointer)(implicit val session: GpuSession) extends Table[GpuTable] {

  import CapsmiLib.{I, check, table}
  import GpuTable._

  GpuTable.cleaner.register(this, new Runnable {
    private val h = handle
    override def run(): Unit = I.capsmi_table_release(h)
  })

  private def wrap(f: com.sun.jna.ptr.PointerByReference => Int): GpuTable = GpuTable(table(f))

  /** (name, physical type, nullable) per column: one call, the plan's schema without running it.  Names
    * are read by walking the NUL terminators (an empty name is a valid column name); a table wider
    * than the first guess is asked again with arrays of its width. */
  private lazy val schema: Seq[(String, Int, Boolean)] = {
    def read(maxCols: Int, nameBytes: Int): Seq[(String, Int, Boolean)] = {
      val names = new Array[Byte](nameBytes)
      val types = new Array[Int](maxCols)
      val nullable = new Array[Int](maxCols)
      val n = new IntByReference
      val rc = I.capsmi_table_schema(handle, n, names, names.length, types, nullable, maxCols)
      if (rc == Capsmi.ERR_ILLEGAL_ARGUMENT && nameBytes < (1 << 28)) return read(maxCols, nameBytes * 4)  // names did not fit
      check(rc)
      if (n.getValue > maxCols) return read(n.getValue, math.max(nameBytes, n.getValue * 256))
      var pos = 0
      (0 until n.getValue).map { i =>
        var end = pos
        while (names(end) != 0) end += 1
        val name = new String(names, pos, end - pos, "UTF-8")
        pos = end + 1
        (name, types(i), nullable(i) != 0)
      }
    }
    read(256, 65536)
  }

  override def physicalColumns: Seq[String] = schema.map(_._1)

  override def columnType: Map[String, CypherType] =
    schema.map { case (n, t, nul) => n -> cypherType(t, nul) }.toMap

  override def size: Long = {
    val v = new LongByReference
    check(I.capsmi_table_size(handle, v))
    v.getValue
  }

  /** DataFrameTable.rows (SparkTable.scala:55-57): exported ExportChunk rows at a time (one host export
    * per column and chunk), so tables above 2^31 rows stream; list columns (Collect results) come
    * back as CypherList. */
  override def rows: Iterator[String => CypherValue] = {
    val n = size
    Iterator.iterate(0L)(_ + ExportChunk).takeWhile(_ < n).flatMap { off =>
      val k = math.min(ExportChunk.toLong, n - off).toInt
      val cols: Seq[(String, Int => CypherValue)] = schema.zipWithIndex.map { case ((name, ty, _), c) =>
        val valid = new com.sun.jna.Memory(math.max(1L, k.toLong))
        if (ty >= Capsmi.LIST) {
          val total = new LongByReference
          check(I.capsmi_table_export_list(handle, c, off, k, null, null, null, 0, total))
          val offs = new com.sun.jna.Memory(8L * (k + 1))
          val vals = new com.sun.jna.Memory(math.max(8L, 8L * total.getValue))
          check(I.capsmi_table_export_list(handle, c, off, k, offs, valid, vals, total.getValue, total))
          val o = offs.getLongArray(0, k + 1)
          val w = vals.getLongArray(0, total.getValue.toInt)
          val v = valid.getByteArray(0, k)
          name -> ((r: Int) => if (v(r) == 0) CypherValue(null)
            else CypherList((o(r) until o(r + 1)).map(i => decode(ty - Capsmi.LIST, w(i.toInt))): _*))
        } else {
          val data = new com.sun.jna.Memory(math.max(8L, 8L * k))
          check(I.capsmi_table_export(handle, c, data, valid, off, k))
          val d = data.getLongArray(0, k)
          val v = valid.getByteArray(0, k)
          name -> ((r: Int) => if (v(r) == 0) CypherValue(null) else decode(ty, d(r)))
        }
      }
      (0 until k).iterator.map(r => cols.map { case (name, get) => name -> get(r) }.toMap)
    }
  }

  override def select(cols: String*): GpuTable = wrap(I.capsmi_select(handle, cols.size, cols.toArray, _))

  override def filter(expr: Expr)(implicit header: RecordHeader, parameters: CypherMap): GpuTable = {
    val prog = ExprCompiler(this, header, parameters).compile(expr)
    wrap(I.capsmi_filter(handle, prog.size, CapsmiLib.exprs(prog), _))
  }

  override def drop(cols: String*): GpuTable = wrap(I.capsmi_drop(handle, cols.size, cols.toArray, _))

  override def join(other: GpuTable, joinType: JoinType, joinCols: (String, String)*): GpuTable =
    wrap(I.capsmi_join(handle, other.handle, joinCode(joinType), joinCols.size, joinCols.map(_._1).toArray,
      joinCols.map(_._2).toArray, _))

  override def unionAll(other: GpuTable): GpuTable = wrap(I.capsmi_union_all(handle, other.handle, _))

  /** SparkTable.scala:94-103: sort keys are expressions; a non-column key is computed first. */
  override def orderBy(sortItems: (Expr, Order)*)(implicit header: RecordHeader, parameters: CypherMap): GpuTable = {
    val (withKeys, keys) = columnsFor(sortItems.map(_._1))
    val desc = sortItems.map { case (_, o) => if (o == Descending) 1 else 0 }.toArray
    val sorted = withKeys.wrap(I.capsmi_order_by(withKeys.handle, keys.size, keys.toArray, desc, _))
    val temps = keys.filterNot(physicalColumns.contains)
    if (temps.isEmpty) sorted else sorted.drop(temps: _*)
  }

  override def skip(n: Long): GpuTable = wrap(I.capsmi_skip(handle, n, _))

  override def limit(n: Long): GpuTable = wrap(I.capsmi_limit(handle, n, _))

  override def distinct: GpuTable = wrap(I.capsmi_distinct(handle, _))

  override def distinct(cols: String*): GpuTable = wrap(I.capsmi_distinct_on(handle, cols.size, cols.toArray, _))

  /** SparkTable.scala:121-188.  Grouping keys are every column the grouped variables own
    * (header.ownedBy, SparkTable.scala:128-133): a node variable groups by its id, label and property
    * columns, which the Aggregate's header keeps (RelationalOperator.scala:345). */
  override def group(by: Set[Var], aggregations: Set[(Aggregator, (String, CypherType))])
    (implicit header: RecordHeader, parameters: CypherMap): GpuTable = {
    val byCols = by.toSeq.flatMap(v => header.ownedBy(v).toSeq.map(header.column)).distinct
    val inputs = aggregations.toSeq.collect {
      case (Avg(e), _) => e
      case (Count(e, _), _) => e
      case (Max(e), _) => e
      case (Min(e), _) => e
      case (Sum(e), _) => e
      case (Collect(e, _), _) => e
    }
    val (withInputs, inCols) = columnsFor(inputs)
    val inputOf = inputs.zip(inCols).toMap
    val specs = aggregations.toSeq.map {
      case (CountStar(_), (out, _)) => (Capsmi.AGG_COUNT_STAR, false, None, out)
      case (Count(e, distinct), (out, _)) => (Capsmi.AGG_COUNT, distinct, Some(inputOf(e)), out)
      case (Min(e), (out, _)) => (Capsmi.AGG_MIN, false, Some(inputOf(e)), out)
      case (Max(e), (out, _)) => (Capsmi.AGG_MAX, false, Some(inputOf(e)), out)
      case (Sum(e), (out, _)) => (Capsmi.AGG_SUM, false, Some(inputOf(e)), out)
      case (Avg(e), (out, _)) => (Capsmi.AGG_AVG, false, Some(inputOf(e)), out)
      case (Collect(e, distinct), (out, _)) => (Capsmi.AGG_COLLECT, distinct, Some(inputOf(e)), out)
      case (other, _) => throw NotImplementedException(s"aggregator $other on the device path")
    }
    withInputs.wrap(I.capsmi_group(withInputs.handle, byCols.size, byCols.toArray, specs.size, CapsmiLib.aggs(specs), _))
  }

  /** SparkTable.scala:69-88: every expression is evaluated against this table; a name that exists
    * is replaced in place. */
  override def withColumns(columns: (Expr, String)*)(implicit header: RecordHeader, parameters: CypherMap): GpuTable = {
    val compiler = ExprCompiler(this, header, parameters)
    val progs = columns.map { case (e, name) => name -> compiler.compile(e) }
    wrap(I.capsmi_with_columns(handle, progs.size, CapsmiLib.exprColumns(progs), _))
  }

  override def withColumnRenamed(oldColumn: String, newColumn: String): GpuTable =
    wrap(I.capsmi_with_column_renamed(handle, oldColumn, newColumn, _))

  /** DataFrameTable.cache (SparkTable.scala:240-246): rows kept once computed; a cached
    * relationship table also keeps the fused layouts built from it. */
  override def cache(): GpuTable = wrap(I.capsmi_cache(handle, _))

  override def show(rows: Int): Unit = {
    val cols = physicalColumns
    println(cols.mkString(" | "))
    this.rows.take(rows).foreach(r => println(cols.map(c => r(c).toCypherString).mkString(" | ")))
  }

  /** Column names holding the values of `exprs` (existing columns, or computed temporaries). */
  private def columnsFor(exprs: Seq[Expr])(implicit header: RecordHeader, parameters: CypherMap): (GpuTable, Seq[String]) = {
    val temps = mutable.ArrayBuffer.empty[(Expr, String)]
    val names = exprs.map { e =>
      if (header.contains(e) && physicalColumns.contains(header.column(e))) header.column(e)
      else {
        val name = s"__capsmi_tmp_${temps.size}"
        temps += e -> name
        name
      }
    }
    (if (temps.isEmpty) this else withColumns(temps: _*), names)
  }
}

/**
  * okapi Expr -> postfix capsmi_expr program, as SparkSQLExprMapper.asSparkSQLExpr
  * (spark-cypher/.../impl/SparkSQLExprMapper.scala:81-312) maps it to a Spark Column: header lookups
  * to column references (:93-104), literals (:107-117), parameters through the session's parameter
  * table (CAPSMI_X_PARAM, :86-92), predicates and arithmetic.  Shapes the device path does not
  * evaluate (string matching, functions, maps, lists other than IN's) raise NotImplementedException.
  */
final case class ExprCompiler(table: GpuTable, header: RecordHeader, parameters: CypherMap) {
  private type Node = (Int, Int, Int, Long)
  private val cols = table.physicalColumns
  private val params = mutable.LinkedHashMap.empty[String, Int]

  def compile(e: Expr): Seq[Node] = {
    val out = mutable.ArrayBuffer.empty[Node]
    go(e, out)
    if (params.nonEmpty) bindParams()
    out
  }

  private def lit(ty: Int, v: Long): Node = (Capsmi.X_LIT, 0, ty, v)

  private def nullOf(ct: CypherType): Node = (Capsmi.X_NULL, physical(ct).map(_ + 1).getOrElse(0), 0, 0L)

  private def physical(ct: CypherType): Option[Int] = ct.material match {
    case CTInteger => Some(Capsmi.I64)
    case CTFloat => Some(Capsmi.F64)
    case CTBoolean => Some(Capsmi.BOOL)
    case CTString => Some(Capsmi.STR)
    case _ => None
  }

  private def column(e: Expr, out: mutable.ArrayBuffer[Node]): Unit = {
    val name = header.column(e)
    val i = cols.indexOf(name)
    out += (if (i >= 0) (Capsmi.X_COL, i, 0, 0L) else nullOf(e.cypherType))
  }

  private def go(e: Expr, out: mutable.ArrayBuffer[Node]): Unit = e match {
    case p: Property if !header.contains(p) => out += nullOf(p.cypherType)
    case p: Param if !header.contains(p) =>
      out += ((Capsmi.X_PARAM, params.getOrElseUpdate(p.name, params.size), 0, 0L))
    case _: Var | _: Param | _: Property | _: HasLabel | _: HasType | _: StartNode | _: EndNode => column(e, out)
    case AliasExpr(inner, _) => go(inner, out)
    case IntegerLit(v) => out += lit(Capsmi.I64, v)
    case StringLit(v) => out += lit(Capsmi.STR, table.session.dictionary.encode(v))
    case b: BoolLit => out += lit(Capsmi.BOOL, if (b.v) 1L else 0L)
    case n: NullLit => out += nullOf(n.cypherType)
    case Equals(l, r) => bin(Capsmi.X_EQ, l, r, out)
    case LessThan(l, r) => bin(Capsmi.X_LT, l, r, out)
    case LessThanOrEqual(l, r) => bin(Capsmi.X_LE, l, r, out)
    case GreaterThan(l, r) => bin(Capsmi.X_GT, l, r, out)
    case GreaterThanOrEqual(l, r) => bin(Capsmi.X_GE, l, r, out)
    case Add(l, r) => bin(Capsmi.X_ADD, l, r, out)
    case Subtract(l, r) => bin(Capsmi.X_SUB, l, r, out)
    case Multiply(l, r) => bin(Capsmi.X_MUL, l, r, out)
    case BitwiseAnd(l, r) => bin(Capsmi.X_BITAND, l, r, out)
    case BitwiseOr(l, r) => bin(Capsmi.X_BITOR, l, r, out)
    case ShiftLeft(v, bits) => bin(Capsmi.X_SHL, v, bits, out)
    case ShiftRightUnsigned(v, bits) => bin(Capsmi.X_SHRU, v, bits, out)
    case Not(x) => go(x, out); out += ((Capsmi.X_NOT, 0, 0, 0L))
    case IsNull(x) => go(x, out); out += ((Capsmi.X_ISNULL, 0, 0, 0L))
    case IsNotNull(x) => go(x, out); out += ((Capsmi.X_ISNOTNULL, 0, 0, 0L))
    case Ands(xs) => nary(Capsmi.X_AND, xs, lit(Capsmi.BOOL, 1L), out)
    case Ors(xs) => nary(Capsmi.X_OR, xs, lit(Capsmi.BOOL, 0L), out)
    case Coalesce(xs) => nary(Capsmi.X_COALESCE, xs, nullOf(CTNull), out)
    case In(lhs, rhs) =>
      go(lhs, out)
      rhs match {
        case ListLit(vs) => vs.foreach(go(_, out)); out += ((Capsmi.X_IN, vs.size, 0, 0L))
        case p: Param if !header.contains(p) =>
          // a list parameter: one IN element that the library expands to the list's values
          out += ((Capsmi.X_PARAM, params.getOrElseUpdate(p.name, params.size), 0, 0L))
          out += ((Capsmi.X_IN, 1, 0, 0L))
        case other => throw NotImplementedException(s"IN over $other on the device path")
      }
    case CaseExpr(alternatives, default) =>
      alternatives.foreach { case (p, v) => go(p, out); go(v, out) }
      default.fold[Unit](out += nullOf(e.cypherType))(go(_, out))
      out += ((Capsmi.X_CASE, alternatives.size, 0, 0L))
    case other => throw NotImplementedException(s"expression $other on the device path")
  }

  private def bin(op: Int, l: Expr, r: Expr, out: mutable.ArrayBuffer[Node]): Unit = {
    go(l, out); go(r, out); out += ((op, 0, 0, 0L))
  }

  private def nary(op: Int, xs: Seq[Expr], empty: Node, out: mutable.ArrayBuffer[Node]): Unit =
    if (xs.isEmpty) out += empty else { xs.foreach(go(_, out)); out += ((op, xs.size, 0, 0L)) }

  /** The parameters this program references, in index order (capsmi_session_set_params). */
  private def bindParams(): Unit = {
    val specs = params.toSeq.sortBy(_._2).map { case (name, _) =>
      parameters.getOrElse(name, throw IllegalArgumentException(s"a value for parameter $$$name", "none"))
    }
    table.session.setParams(specs)
  }
}
