/*
 * GpuRowEncoder — the Java drop-in for the MI355X row codec (libfury_row.so through
 * libfury_row_jni.so).  NOT COMPILED IN THIS REPOSITORY: the build image has no JDK and no
 * Maven (DESIGN.md §1); it is the binding a maintainer adds next to
 * java/fury-format/src/main/java/org/apache/fury/format/encoder/Encoders.java.
 *
 * Per-object API: identical to RowEncoder<T> (RowEncoder.java:26-32, Encoder.java:31-40) — it
 * delegates to Encoders.bean(cls), so existing callers (RowSuite.java:100-126, FMTT/*) keep their
 * exact bytes and exceptions.
 * Batch API: Arrow columns (a VectorSchemaRoot, as ArrowWriter produces them, ArrowWriter.java:
 * 55-99) <-> packed rows in off-heap MemoryBuffers, through fury_row_encode_host /
 * fury_row_decode_host, and fury_decode_host_prepare / _execute for nested beans
 * (include/fury_row.h): the buffers' addresses cross JNI, the bytes cross PCIe inside the native
 * call, the rows are bit-identical to toRow(obj) for every object.
 */
package org.apache.fury.format.encoder;

import java.util.ArrayList;
import java.util.List;
import org.apache.arrow.memory.ArrowBuf;
import org.apache.arrow.vector.BaseVariableWidthVector;
import org.apache.arrow.vector.BitVector;
import org.apache.arrow.vector.FieldVector;
import org.apache.arrow.vector.VectorSchemaRoot;
import org.apache.arrow.vector.complex.ListVector;
import org.apache.arrow.vector.complex.MapVector;
import org.apache.arrow.vector.complex.StructVector;
import org.apache.arrow.vector.types.pojo.Field;
import org.apache.arrow.vector.types.pojo.Schema;
import org.apache.fury.format.row.binary.BinaryRow;
import org.apache.fury.format.type.DataTypes;
import org.apache.fury.memory.MemoryBuffer;

public final class GpuRowEncoder<T> implements RowEncoder<T> {
  static {
    System.loadLibrary("fury_row_jni");
  }

  private final RowEncoder<T> cpu;
  private final long schemaHandle;      // fury_schema*, freed by close()
  private final int device;
  private final boolean nested;         // nested beans / maps / lists of var elements
  private final int numNodes;

  public GpuRowEncoder(Class<T> beanClass, int device) {
    this.cpu = Encoders.bean(beanClass);
    this.device = device;
    List<String> names = new ArrayList<>();
    List<Integer> meta = new ArrayList<>();       // per node: typeId, nullable, numChildren
    for (Field f : cpu.schema().getFields()) {
      flattenField(f, names, meta);
    }
    int[] m = new int[meta.size()];
    for (int i = 0; i < m.length; i++) {
      m[i] = meta.get(i);
    }
    this.schemaHandle =
        nativeSchemaCreate(names.toArray(new String[0]), m, cpu.schema().getFields().size());
    this.numNodes = nativeSchemaNumNodes(schemaHandle);
    boolean deep = false;
    for (Field f : cpu.schema().getFields()) {
      deep |= isNested(f);
    }
    this.nested = deep;
  }

  private static boolean isNested(Field f) {
    org.apache.arrow.vector.types.pojo.ArrowType t = f.getType();
    if (t instanceof org.apache.arrow.vector.types.pojo.ArrowType.Struct
        || t instanceof org.apache.arrow.vector.types.pojo.ArrowType.Map) {
      return true;
    }
    if (t instanceof org.apache.arrow.vector.types.pojo.ArrowType.List) {
      Field e = f.getChildren().get(0);
      return DataTypes.getTypeWidth(e.getType()) < 0 || isNested(e);
    }
    return false;
  }

  // ---- RowEncoder<T>: the reference implementation, unchanged ----------------------------
  @Override public Schema schema() { return cpu.schema(); }
  @Override public BinaryRow toRow(T obj) { return cpu.toRow(obj); }
  @Override public T fromRow(BinaryRow row) { return cpu.fromRow(row); }
  @Override public byte[] encode(T obj) { return cpu.encode(obj); }
  @Override public void encode(MemoryBuffer buffer, T obj) { cpu.encode(buffer, obj); }
  @Override public T decode(byte[] bytes) { return cpu.decode(bytes); }
  @Override public T decode(MemoryBuffer buffer) { return cpu.decode(buffer); }

  // ---- batch path --------------------------------------------------------------------------
  /**
   * Encodes root.getRowCount() rows into the off-heap buffer `rows` (row i at
   * rowOffsets[i], int64 little-endian, nrows + 1 entries; for all-fixed-width schemas row i is at
   * i * fixedSize and rowOffsets may be null).  Returns the row bytes written.  Throws
   * IndexOutOfBoundsException-family errors exactly where fury_status says.
   */
  public long encodeBatch(VectorSchemaRoot root, MemoryBuffer rows, MemoryBuffer rowOffsets) {
    checkOffHeap(rows);
    long[] desc = describe(root, false);
    return nativeEncodeHost(schemaHandle, desc, root.getRowCount(), rows.getUnsafeAddress(),
        rows.size(), rowOffsets == null ? 0 : addressOf(rowOffsets), device);
  }

  /** Decodes nrows rows into `out`.  Flat schemas: vectors allocated by the caller for nrows
   * values and, for strings / lists, enough payload capacity.  Schemas with nested beans, maps or
   * lists of structs / strings: the vectors are (re)allocated here from the per-node sizes the
   * device counts (fury_decode_host_prepare), then filled (fury_decode_host_execute).  Sets the
   * value counts. */
  public void decodeBatch(MemoryBuffer rows, MemoryBuffer rowOffsets, int nrows,
                          VectorSchemaRoot out) {
    checkOffHeap(rows);
    long offs = rowOffsets == null ? 0 : addressOf(rowOffsets);
    if (nested) {
      decodeNested(rows.getUnsafeAddress(), offs, nrows, out);
      return;
    }
    long[] desc = describe(out, true);
    nativeDecodeHost(schemaHandle, rows.getUnsafeAddress(), offs, nrows, desc, device);
    for (FieldVector v : out.getFieldVectors()) {       // offsets are written: no hole filling
      if (v instanceof BaseVariableWidthVector) {
        ((BaseVariableWidthVector) v).setLastSet(nrows - 1);
      } else if (v instanceof ListVector) {
        ((ListVector) v).setLastSet(nrows - 1);
      }
    }
    out.setRowCount(nrows);
  }

  private void decodeNested(long rows, long rowOffsets, int nrows, VectorSchemaRoot out) {
    long[] counts = new long[2 * numNodes];             // per node: entries, payload bytes
    long plan = nativeDecodeHostPrepare(schemaHandle, rows, rowOffsets, nrows, counts, device);
    try {
      List<FieldVector> nodes = breadthFirst(out);      // the C ABI's node order
      for (int i = 0; i < nodes.size(); i++) {          // parents before children
        FieldVector v = nodes.get(i);
        int entries = (int) counts[2 * i];
        if (v instanceof BaseVariableWidthVector) {
          ((BaseVariableWidthVector) v).allocateNew(Math.max(counts[2 * i + 1], 1), entries);
        } else {
          v.setInitialCapacity(entries);
          v.allocateNew();
        }
      }
      nativeDecodeHostExecute(schemaHandle, plan, describe(out, true));
      // A MapVector's entries struct is not a schema node (fury_row.h): the native side writes
      // no validity for it, and every entry of a map is a defined (key, value) struct, as the
      // reference's MapWriter marks them through startEntry / endEntry (ArrowWriter.java:623-630).
      for (int i = 0; i < nodes.size(); i++) {
        FieldVector v = nodes.get(i);
        if (v instanceof MapVector) {
          int entries = (int) counts[2 * i];
          int children = entries == 0 ? 0 : v.getOffsetBuffer().getInt((long) entries * 4);
          StructVector kv = (StructVector) ((MapVector) v).getDataVector();
          for (int j = 0; j < children; j++) {
            kv.setIndexDefined(j);
          }
          kv.setValueCount(children);
        }
      }
      for (int i = nodes.size() - 1; i >= 0; i--) {     // children first
        FieldVector v = nodes.get(i);
        int entries = (int) counts[2 * i];
        if (v instanceof BaseVariableWidthVector) {
          ((BaseVariableWidthVector) v).setLastSet(entries - 1);
        } else if (v instanceof ListVector) {
          ((ListVector) v).setLastSet(entries - 1);
        }
        v.setValueCount(entries);
      }
      out.setRowCount(nrows);
    } finally {
      nativeDecodePlanDestroy(plan);
    }
  }

  /** Vectors in the schema-node order of fury_row.h: top-level fields, then every node's
   * children (LIST: data vector; STRUCT: fields; MAP: key, value -- the entries struct skipped). */
  private static List<FieldVector> breadthFirst(VectorSchemaRoot root) {
    List<FieldVector> q = new ArrayList<>(root.getFieldVectors());
    for (int i = 0; i < q.size(); i++) {
      FieldVector v = q.get(i);
      if (v instanceof MapVector) {
        StructVector entries = (StructVector) ((MapVector) v).getDataVector();
        q.add((FieldVector) entries.getChildByOrdinal(0));
        q.add((FieldVector) entries.getChildByOrdinal(1));
      } else if (v instanceof ListVector) {
        q.add(((ListVector) v).getDataVector());
      } else if (v instanceof StructVector) {
        q.addAll(((StructVector) v).getChildrenFromFields());
      }
    }
    return q;
  }

  public void close() {
    nativeSchemaDestroy(schemaHandle);
  }

  // ---- pinned host memory (fury_host_alloc / fury_host_register) ---------------------------
  // encodeBatch / decodeBatch of fixed-width beans run the kernels directly on host memory when
  // every buffer of the call is pinned (no staging through HBM; both PCIe directions busy).

  /** Off-heap memory the GPU reaches directly (hipHostMalloc); release with freePinned. */
  public static MemoryBuffer allocatePinned(int bytes) {
    return MemoryBuffer.fromNativeAddress(nativeHostAlloc(bytes), bytes);
  }

  public static void freePinned(MemoryBuffer buffer) {
    nativeHostFree(buffer.getUnsafeAddress());
  }

  /** Pins existing off-heap memory in place (hipHostRegister), e.g. a long-lived ArrowBuf. */
  public static void pin(long address, long bytes) {
    nativeHostRegister(address, bytes);
  }

  public static void unpin(long address) {
    nativeHostUnregister(address);
  }

  static long hostAlloc(long bytes) {
    return nativeHostAlloc(bytes);
  }

  static void hostFree(long address) {
    nativeHostFree(address);
  }

  // ---- column descriptors: 5 longs per node in pre-order ----------------------------------
  // {values address, validity address, offsets address, values capacity, number of children};
  // a MAP's children are its keys and values vectors (the "entries" struct is skipped, as in
  // fury_row.h's fury_column).
  private static long[] describe(VectorSchemaRoot root, boolean decode) {
    List<Long> d = new ArrayList<>();
    for (FieldVector v : root.getFieldVectors()) {
      describe(v, decode, d);
    }
    long[] out = new long[d.size()];
    for (int i = 0; i < out.length; i++) {
      out[i] = d.get(i);
    }
    return out;
  }

  private static void describe(FieldVector v, boolean decode, List<Long> d) {
    boolean nullable = v.getField().isNullable();
    ArrowBuf validity = v.getValidityBuffer();
    List<FieldVector> kids = new ArrayList<>();
    long values = 0, offsets = 0, capacity = 0;
    if (v instanceof MapVector) {
      StructVector entries = (StructVector) ((MapVector) v).getDataVector();
      kids.add((FieldVector) entries.getChildByOrdinal(0));
      kids.add((FieldVector) entries.getChildByOrdinal(1));
      offsets = v.getOffsetBuffer().memoryAddress();
    } else if (v instanceof ListVector) {
      kids.add(((ListVector) v).getDataVector());
      offsets = v.getOffsetBuffer().memoryAddress();
    } else if (v instanceof StructVector) {
      kids.addAll(((StructVector) v).getChildrenFromFields());
    } else {
      values = v.getDataBuffer().memoryAddress();
      capacity = v.getDataBuffer().capacity();
      if (v instanceof BaseVariableWidthVector) {
        offsets = v.getOffsetBuffer().memoryAddress();
      }
    }
    d.add(values);
    d.add(nullable && (decode || v.getNullCount() > 0) ? validity.memoryAddress() : 0L);
    d.add(offsets);
    d.add(capacity);
    d.add((long) kids.size());
    for (FieldVector k : kids) {
      describe(k, decode, d);
    }
  }

  private static void flattenField(Field f, List<String> names, List<Integer> meta) {
    List<Field> kids = f.getChildren();
    if (f.getType() instanceof org.apache.arrow.vector.types.pojo.ArrowType.Map) {
      kids = kids.get(0).getChildren();          // entries struct -> (key, value)
    }
    names.add(f.getName());
    meta.add((int) DataTypes.getTypeIdValue(f.getType()));
    meta.add(f.isNullable() ? 1 : 0);
    meta.add(kids.size());
    for (Field k : kids) {
      flattenField(k, names, meta);
    }
  }

  private static long addressOf(MemoryBuffer b) {
    checkOffHeap(b);
    return b.getUnsafeAddress();
  }

  private static void checkOffHeap(MemoryBuffer b) {
    if (!b.isOffHeap()) {
      throw new IllegalArgumentException("batch buffers must be off-heap (DirectByteBuffer)");
    }
  }

  private static native long nativeSchemaCreate(String[] names, int[] meta, int numTopFields);
  private static native void nativeSchemaDestroy(long schema);
  private static native long nativeEncodeHost(long schema, long[] columns, long nrows, long rows,
                                              long rowsCapacity, long rowOffsets, int device);
  private static native void nativeDecodeHost(long schema, long rows, long rowOffsets, long nrows,
                                              long[] columns, int device);
  private static native int nativeSchemaNumNodes(long schema);
  private static native long nativeDecodeHostPrepare(long schema, long rows, long rowOffsets,
                                                     long nrows, long[] counts, int device);
  private static native void nativeDecodeHostExecute(long schema, long plan, long[] columns);
  private static native void nativeDecodePlanDestroy(long plan);
  private static native long nativeHostAlloc(long bytes);
  private static native void nativeHostFree(long address);
  private static native void nativeHostRegister(long address, long bytes);
  private static native void nativeHostUnregister(long address);
}
