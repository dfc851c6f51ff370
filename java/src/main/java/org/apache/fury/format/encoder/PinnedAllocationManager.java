/*
 * Arrow allocation manager over pinned host memory (include/fury_row.h fury_host_alloc):
 * vectors of a RootAllocator built with
 *   RootAllocator.configBuilder().allocationManagerFactory(PinnedAllocationManager.FACTORY)
 * live in memory the GPU reaches directly, so GpuRowEncoder.encodeBatch / decodeBatch of
 * fixed-width beans on them run the kernels on host memory with no staging copy.
 */
package org.apache.fury.format.encoder;

import org.apache.arrow.memory.AllocationManager;
import org.apache.arrow.memory.ArrowBuf;
import org.apache.arrow.memory.BufferAllocator;
import org.apache.arrow.memory.ReferenceManager;

public final class PinnedAllocationManager extends AllocationManager {
  public static final AllocationManager.Factory FACTORY =
      new AllocationManager.Factory() {
        @Override
        public AllocationManager create(BufferAllocator accountingAllocator, long size) {
          return new PinnedAllocationManager(accountingAllocator, size);
        }

        @Override
        public ArrowBuf empty() {
          return EMPTY;
        }
      };

  // zero capacity at address 0, as Arrow's own managers do: loading the class needs neither the
  // native library nor a GPU, and nothing is allocated that would never be freed
  private static final ArrowBuf EMPTY = new ArrowBuf(ReferenceManager.NO_OP, null, 0, 0);

  private final long address;
  private final long size;

  private PinnedAllocationManager(BufferAllocator accountingAllocator, long size) {
    super(accountingAllocator);
    this.size = size;
    this.address = GpuRowEncoder.hostAlloc(Math.max(size, 1));
  }

  @Override
  public long getSize() {
    return size;
  }

  @Override
  protected long memoryAddress() {
    return address;
  }

  @Override
  protected void release0() {
    GpuRowEncoder.hostFree(address);
  }
}
