/*
 * JNA binding of libcapsmi's C ABI (include/capsmi.h) for the CAPS JVM side.
 *
 * This is the source a CAPS maintainer adds next to spark-cypher to run the relational pattern-
 * matching path on MI355X.  It is NOT compiled in this repository (the image has no JVM; see
 * INTEGRATION.md).  Every declaration below mirrors one prototype of include/capsmi.h; struct field
 * order is the C layout.  The same ABI is exercised from Python ctypes in
 * cypher-for-apache-spark_amd/capsmi/_lib.py, whose tests/test_abi.py checks that every symbol is
 * exported.
 */
package org.opencypher.capsmi

import com.sun.jna.ptr.{DoubleByReference, IntByReference, LongByReference, PointerByReference}
import com.sun.jna.{Callback, Library, Memory, Native, Pointer, Structure}
import org.opencypher.okapi.impl.exception.{IllegalArgumentException, IllegalStateException, NotImplementedException, UnsupportedOperationException}

/** Constants of include/capsmi.h. */
object Capsmi {
  // status codes (capsmi_status)
  final val OK = 0
  final val ERR_ILLEGAL_ARGUMENT = 1
  final val ERR_NOT_IMPLEMENTED = 2
  final val ERR_UNSUPPORTED = 3
  final val ERR_DEVICE = 4
  final val ERR_OUT_OF_MEMORY = 5
  final val ERR_INTERNAL = 6

  // physical column types
  final val I64 = 0  // CTInteger, entity ids
  final val BOOL = 1 // CTBoolean, label / relationship-type flags
  final val F64 = 2  // CTFloat
  final val STR = 3  // CTString as an order-preserving dictionary code
  final val LIST = 8 // CTList(elem): LIST + elem type (Collect results; read with capsmi_table_export_list)
  // host widths widened at ingest (DataFrameOps.withCypherCompatibleTypes)
  final val IN_I32 = 16
  final val IN_I16 = 17
  final val IN_I8 = 18
  final val IN_F32 = 19
  final val IN_BOOL8 = 20

  // expression opcodes (postfix programs, capsmi_expr)
  final val X_COL = 0
  final val X_LIT = 1
  final val X_NULL = 2
  final val X_EQ = 3
  final val X_NEQ = 4
  final val X_LT = 5
  final val X_LE = 6
  final val X_GT = 7
  final val X_GE = 8
  final val X_NOT = 9
  final val X_AND = 10
  final val X_OR = 11
  final val X_ISNULL = 12
  final val X_ISNOTNULL = 13
  final val X_IN = 14
  final val X_ADD = 15
  final val X_SUB = 16
  final val X_MUL = 17
  final val X_NEG = 18
  final val X_COALESCE = 19
  final val X_BITAND = 20
  final val X_BITOR = 21
  final val X_SHL = 22
  final val X_SHRU = 23
  final val X_CASE = 24
  final val X_PARAM = 25

  // join types (JoinType of RelationalPlanner; SparkTable.scala:205-229)
  final val JOIN_INNER = 0
  final val JOIN_LEFT_OUTER = 1
  final val JOIN_RIGHT_OUTER = 2
  final val JOIN_FULL_OUTER = 3
  final val JOIN_CROSS = 4

  // aggregates (SparkTable.scala:121-188)
  final val AGG_COUNT_STAR = 0
  final val AGG_COUNT = 1
  final val AGG_MIN = 2
  final val AGG_MAX = 3
  final val AGG_SUM = 4
  final val AGG_AVG = 5
  final val AGG_COLLECT = 6 // sort_array(collect_list / collect_set)

  // multi-GPU: collectives the library asks the host for, shard layouts (capsmi_graph_distribute)
  final val COLL_ALL_GATHER = 0
  final val COLL_ALL_REDUCE_SUM = 1
  final val COLL_ALL_REDUCE_MAX = 2
  final val COLL_ALL_TO_ALL_V = 3 // send / recv point to CapsmiCollVec descriptors, count = world size
  final val COLL_U32 = 100
  final val NODES_REPLICATED = 0
  final val NODES_OWNED = 1
  final val RELS_BY_SOURCE = 0
  final val RELS_BY_TARGET = 1
}

@Structure.FieldOrder(Array("name", "type", "data", "valid"))
class ColDesc extends Structure {
  var name: String = _
  var `type`: Int = 0
  var data: Pointer = _
  var valid: Pointer = _
}

@Structure.FieldOrder(Array("op", "arg", "type", "reserved", "ival"))
class CapsmiExpr extends Structure {
  var op: Int = 0
  var arg: Int = 0
  var `type`: Int = 0
  var reserved: Int = 0
  var ival: Long = 0L
}

@Structure.FieldOrder(Array("name", "nnodes", "prog"))
class CapsmiExprColumn extends Structure {
  var name: String = _
  var nnodes: Int = 0
  var prog: Pointer = _
}

@Structure.FieldOrder(Array("kind", "distinct", "input", "output"))
class CapsmiAgg extends Structure {
  var kind: Int = 0
  var distinct: Int = 0
  var input: String = _
  var output: String = _
}

@Structure.FieldOrder(Array("ival", "is_null", "reserved"))
class CapsmiValue extends Structure {
  var ival: Long = 0L
  var is_null: Int = 0
  var reserved: Int = 0
}

@Structure.FieldOrder(Array("type", "is_list", "count", "reserved", "values"))
class CapsmiParam extends Structure {
  var `type`: Int = 0
  var is_list: Int = 0
  var count: Int = 0
  var reserved: Int = 0
  var values: Pointer = _
}

/** capsmi_coll_vec: an ALL_TO_ALL_V side -- device data in rank-major segments, host counts per rank
  * (inside the CollectiveFn: `Structure.newInstance(classOf[CapsmiCollVec], ptr)` then `read()`). */
@Structure.FieldOrder(Array("data", "counts"))
class CapsmiCollVec extends Structure {
  var data: Pointer = _
  var counts: Pointer = _
}

/** capsmi_collective_fn: one collective on the session's stream (e.g. an RCCL communicator the executor
  * holds, over xGMI); 0 on success. */
trait CollectiveFn extends Callback {
  def invoke(ctx: Pointer, op: Int, send: Pointer, recv: Pointer, count: Long, dtype: Int): Int
}

/** capsmi_intern_fn: strings of a CSV column handed, in row order, to the session's dictionary. */
trait InternFn extends Callback {
  def invoke(ctx: Pointer, s: Pointer, n: Long): Long
}

trait CapsmiLib extends Library {
  def capsmi_last_error(buf: Array[Byte], n: Long): Long

  // sessions
  def capsmi_session_create(device: Int, out: PointerByReference): Int
  def capsmi_session_destroy(s: Pointer): Int
  def capsmi_session_set_stream(s: Pointer, hipStream: Pointer): Int
  def capsmi_session_use_stream(s: Pointer, hipStream: Pointer): Int
  def capsmi_session_sync(s: Pointer): Int
  // session configuration (CAPSMI_* knobs; read from the environment once, at create): name, value (null = default)
  def capsmi_session_set_config(s: Pointer, name: String, value: String): Int
  def capsmi_config_check(name: String, value: String): Int
  def capsmi_session_set_profiling(s: Pointer, enabled: Int): Int
  def capsmi_session_set_profiling_names(s: Pointer, names: String): Int
  def capsmi_session_kernel_time(s: Pointer, name: String, launches: LongByReference, totalMs: DoubleByReference): Int
  def capsmi_session_kernel_bytes(s: Pointer, name: String, bytes: DoubleByReference): Int
  def capsmi_session_set_fused(s: Pointer, enabled: Int): Int
  def capsmi_session_set_params(s: Pointer, nparams: Int, params: CapsmiParam): Int
  def capsmi_session_route_count(s: Pointer, name: String, count: LongByReference): Int
  def capsmi_session_set_unrouted_limit(s: Pointer, maxBytes: Long): Int
  def capsmi_session_set_csv_partitioning(s: Pointer, defaultParallelism: Long, maxPartitionBytes: Long,
                                          openCostBytes: Long): Int

  // multi-GPU (one process per GPU): rank view, shards of a distributed graph
  def capsmi_session_set_ranks(s: Pointer, rank: Int, world: Int, fn: CollectiveFn, ctx: Pointer): Int
  def capsmi_graph_distribute(s: Pointer, idLo: Long, idHi: Long, nnodes: Int, nodes: Array[Pointer], nodeMode: Int,
                              nrels: Int, rels: Array[Pointer], relMode: Int): Int
  def capsmi_owned_rows(s: Pointer, t: Pointer, col: String, idLo: Long, idHi: Long, out: PointerByReference): Int
  def capsmi_table_partitioned(t: Pointer, out: IntByReference): Int
  def capsmi_id_owner(idLo: Long, idHi: Long, world: Int, id: Long, owner: IntByReference, denseId: LongByReference): Int

  // tables
  def capsmi_table_from_host(s: Pointer, ncols: Int, cols: ColDesc, nrows: Long, out: PointerByReference): Int
  def capsmi_table_from_device(s: Pointer, ncols: Int, cols: ColDesc, nrows: Long, out: PointerByReference): Int
  def capsmi_table_retain(t: Pointer): Int
  def capsmi_table_release(t: Pointer): Int
  def capsmi_table_size(t: Pointer, out: LongByReference): Int
  def capsmi_table_num_columns(t: Pointer, out: IntByReference): Int
  def capsmi_table_column_name(t: Pointer, col: Int, buf: Array[Byte], n: Long): Int
  def capsmi_table_column_type(t: Pointer, col: Int, out: IntByReference): Int
  def capsmi_table_column_index(t: Pointer, name: String, out: IntByReference): Int
  def capsmi_table_column_nullable(t: Pointer, col: Int, out: IntByReference): Int
  def capsmi_table_schema(t: Pointer, ncols: IntByReference, names: Array[Byte], namesLen: Long, types: Array[Int],
                          nullable: Array[Int], maxCols: Int): Int
  def capsmi_table_export(t: Pointer, col: Int, hostData: Pointer, hostValid: Pointer, offset: Long, n: Long): Int
  def capsmi_table_export_list(t: Pointer, col: Int, offset: Long, n: Long, hostOffsets: Pointer, hostValid: Pointer,
                               hostValues: Pointer, valuesCap: Long, nvalues: LongByReference): Int
  def capsmi_table_column_device_ptr(t: Pointer, col: Int, data: PointerByReference, valid: PointerByReference): Int
  def capsmi_table_fingerprint(t: Pointer, ncols: Int, cols: Array[String], count: LongByReference,
                               sum: LongByReference, xr: LongByReference): Int

  // entity tables (EntityTable.verify, CAPSTable relType flattening)
  def capsmi_node_table(t: Pointer, idCol: String, nlabels: Int, labelCols: Array[String], out: PointerByReference): Int
  def capsmi_rel_table(t: Pointer, idCol: String, srcCol: String, dstCol: String, ntypes: Int, typeCols: Array[String],
                       out: PointerByReference): Int
  def capsmi_graph_compact(s: Pointer, nnodes: Int, nodes: Array[Pointer], nrels: Int, rels: Array[Pointer],
                           denseIds: LongByReference): Int
  def capsmi_table_entity(t: Pointer, kind: IntByReference, idLo: LongByReference, idHi: LongByReference): Int
  def capsmi_flatten_rel_types(t: Pointer, typeCol: String, ntypes: Int, typeCodes: Array[Long], outCols: Array[String],
                               out: PointerByReference): Int

  // Table[T] operators (lazy plans; Table.scala:43-176)
  def capsmi_cache(t: Pointer, out: PointerByReference): Int
  def capsmi_select(t: Pointer, ncols: Int, cols: Array[String], out: PointerByReference): Int
  def capsmi_filter(t: Pointer, nnodes: Int, prog: CapsmiExpr, out: PointerByReference): Int
  def capsmi_drop(t: Pointer, ncols: Int, cols: Array[String], out: PointerByReference): Int
  def capsmi_join(l: Pointer, r: Pointer, joinType: Int, npairs: Int, lcols: Array[String], rcols: Array[String],
                  out: PointerByReference): Int
  def capsmi_union_all(a: Pointer, b: Pointer, out: PointerByReference): Int
  def capsmi_order_by(t: Pointer, nkeys: Int, cols: Array[String], descending: Array[Int], out: PointerByReference): Int
  def capsmi_skip(t: Pointer, n: Long, out: PointerByReference): Int
  def capsmi_limit(t: Pointer, n: Long, out: PointerByReference): Int
  def capsmi_distinct(t: Pointer, out: PointerByReference): Int
  def capsmi_distinct_on(t: Pointer, ncols: Int, cols: Array[String], out: PointerByReference): Int
  def capsmi_group(t: Pointer, nby: Int, by: Array[String], naggs: Int, aggs: CapsmiAgg, out: PointerByReference): Int
  def capsmi_with_columns(t: Pointer, ncols: Int, cols: CapsmiExprColumn, out: PointerByReference): Int
  def capsmi_with_column_renamed(t: Pointer, oldName: String, newName: String, out: PointerByReference): Int

  // explicit graph entry points (the lazy plans reach the same kernels through the recogniser)
  def capsmi_bitmap_create(s: Pointer, idLo: Long, idHi: Long, out: PointerByReference): Int
  def capsmi_bitmap_add_scan(b: Pointer, nodes: Pointer, idCol: String, nnodes: Int, pred: CapsmiExpr): Int
  def capsmi_bitmap_stats(b: Pointer, setBits: LongByReference, uniqueRows: IntByReference): Int
  def capsmi_bitmap_release(b: Pointer): Int
  def capsmi_expand_filter(s: Pointer, rels: Pointer, srcCol: String, dstCol: String, srcOk: Pointer, dstOk: Pointer,
                           nout: Int, outCols: Array[String], outNames: Array[String], out: PointerByReference): Int
  def capsmi_two_hop_count(s: Pointer, nrels: Int, rels: Array[Pointer], srcCol: String, dstCol: String, a: Pointer,
                           b: Pointer, c: Pointer, outRows: LongByReference): Int
  def capsmi_two_hop_count_distinct(s: Pointer, nrels: Int, rels: Array[Pointer], srcCol: String, dstCol: String,
                                    a: Pointer, b: Pointer, c: Pointer, outDistinct: LongByReference): Int
  def capsmi_triangle_count(s: Pointer, nrels: Int, rels: Array[Pointer], srcCol: String, dstCol: String, nOk: Pointer,
                            outRows: LongByReference): Int
  def capsmi_undirected_count(s: Pointer, nrels: Int, rels: Array[Pointer], srcCol: String, dstCol: String, hops: Int,
                              a: Pointer, b: Pointer, c: Pointer, kind: Int, out: LongByReference): Int
  def capsmi_var_length_count(s: Pointer, nrels: Int, rels: Array[Pointer], srcCol: String, dstCol: String, a: Pointer,
                              b: Pointer, lower: Int, upper: Int, idName: String, countName: String,
                              out: PointerByReference): Int

  // ingest (EdgeListDataSource / FSGraphSource CSV)
  def capsmi_read_csv(s: Pointer, nfiles: Int, paths: Array[String], delimiter: Byte, comment: Byte, ncols: Int,
                      names: Array[String], types: Array[Int], intern: InternFn, ctx: Pointer, rowIdCol: String,
                      out: PointerByReference): Int
}

object CapsmiLib {
  lazy val I: CapsmiLib = Native.load("capsmi", classOf[CapsmiLib])

  /** Status codes to okapi exceptions (okapi-api/.../impl/exception/InternalException.scala:34-59). */
  def check(rc: Int): Unit = if (rc != Capsmi.OK) {
    val buf = new Array[Byte](4096)
    I.capsmi_last_error(buf, buf.length)
    val msg = new String(buf.takeWhile(_ != 0), "UTF-8")
    rc match {
      case Capsmi.ERR_ILLEGAL_ARGUMENT => throw IllegalArgumentException("a valid argument", msg)
      case Capsmi.ERR_NOT_IMPLEMENTED => throw NotImplementedException(msg)
      case Capsmi.ERR_UNSUPPORTED => throw UnsupportedOperationException(msg)
      case _ => throw IllegalStateException(s"capsmi status $rc: $msg")
    }
  }

  /** A new table handle from a call that writes one (the result is owned by the caller). */
  def table(f: PointerByReference => Int): Pointer = {
    val out = new PointerByReference
    check(f(out))
    out.getValue
  }

  /** Contiguous native arrays of structures: JNA passes the first element by reference. */
  def exprs(prog: Seq[(Int, Int, Int, Long)]): CapsmiExpr = {
    val arr = new CapsmiExpr().toArray(math.max(1, prog.size)).asInstanceOf[Array[CapsmiExpr]]
    prog.zipWithIndex.foreach { case ((op, arg, ty, ival), i) =>
      arr(i).op = op; arr(i).arg = arg; arr(i).`type` = ty; arr(i).ival = ival; arr(i).write()
    }
    arr(0)
  }

  def exprColumns(cols: Seq[(String, Seq[(Int, Int, Int, Long)])]): CapsmiExprColumn = {
    val arr = new CapsmiExprColumn().toArray(math.max(1, cols.size)).asInstanceOf[Array[CapsmiExprColumn]]
    cols.zipWithIndex.foreach { case ((name, prog), i) =>
      val p = exprs(prog)
      arr(i).name = name; arr(i).nnodes = prog.size; arr(i).prog = p.getPointer; arr(i).write()
    }
    arr(0)
  }

  def aggs(as: Seq[(Int, Boolean, Option[String], String)]): CapsmiAgg = {
    val arr = new CapsmiAgg().toArray(math.max(1, as.size)).asInstanceOf[Array[CapsmiAgg]]
    as.zipWithIndex.foreach { case ((kind, distinct, input, output), i) =>
      arr(i).kind = kind; arr(i).distinct = if (distinct) 1 else 0; arr(i).input = input.orNull; arr(i).output = output
      arr(i).write()
    }
    arr(0)
  }

  /** Native copy of a host column (int64 words) and its validity bytes. */
  def words(values: Array[Long]): Memory = {
    val m = new Memory(math.max(8L, 8L * values.length))
    m.write(0, values, 0, values.length)
    m
  }

  def bytes(values: Array[Byte]): Memory = {
    val m = new Memory(math.max(1L, values.length.toLong))
    m.write(0, values, 0, values.length)
    m
  }
}
