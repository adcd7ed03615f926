/*
 * EngineDecodedLog -- the decode side of DeterminantEncoder (DeterminantEncoder.java:28-65)
 * over one log, with the record boundaries found on the GPU in one batch.
 *
 * SimpleDeterminantEncoder.decodeNext (:78-112) walks the log one record at a time; the
 * length of a record is known only once its tag (and, for TimerTrigger / SourceCheckpoint,
 * a field) was read, so the walk is sequential.  Here the whole log is decoded by the
 * engine (clg_decode_host: record offsets, tags and fields in one pass), and next() hands
 * the records out in order.  Each Determinant object is still materialised by the
 * reference's own per-type reader (SimpleDeterminantEncoder.decodeXDeterminant(buf, reuse))
 * positioned at the record's first field, so objects, DeterminantPool reuse and the
 * Serializable path (ObjectInputStream, SimpleDeterminantEncoder.java:333-341) are the
 * reference's.
 *
 * A log the engine reports an error for (a corrupt tag, an out-of-range ordinal, a negative
 * length, a truncated record, a Serializable stream the engine does not accept) is replayed
 * by the engine up to the failing record; from that record on the reference's own
 * decodeNext takes over on the same buffer, so the exception it throws -- or, for a
 * malformed Serializable stream, its print-and-continue behaviour (:335-339) -- is exactly
 * the reference's.
 *
 * Source-only: this container has no JDK, so the binding is not compiled here.
 */
package org.apache.flink.runtime.causal.engine;

import org.apache.flink.runtime.causal.determinant.BufferBuiltDeterminant;
import org.apache.flink.runtime.causal.determinant.Determinant;
import org.apache.flink.runtime.causal.determinant.DeterminantEncoder;
import org.apache.flink.runtime.causal.determinant.IgnoreCheckpointDeterminant;
import org.apache.flink.runtime.causal.determinant.OrderDeterminant;
import org.apache.flink.runtime.causal.determinant.RNGDeterminant;
import org.apache.flink.runtime.causal.determinant.SerializableDeterminant;
import org.apache.flink.runtime.causal.determinant.SourceCheckpointDeterminant;
import org.apache.flink.runtime.causal.determinant.TimerTriggerDeterminant;
import org.apache.flink.runtime.causal.determinant.TimestampDeterminant;
import org.apache.flink.runtime.causal.recovery.DeterminantPool;
import org.apache.flink.shaded.netty4.io.netty.buffer.ByteBuf;
import org.apache.flink.shaded.netty4.io.netty.buffer.Unpooled;

import java.nio.ByteBuffer;
import java.nio.ByteOrder;

import static org.apache.flink.runtime.causal.engine.ClonosEngine.*;

public final class EngineDecodedLog {

	private final ByteBuf log;
	private final int base; // readerIndex of the log when decoded (record offsets are relative to it)
	private final DeterminantEncoder encoder;
	private final int nRec;
	private final ByteBuffer recOff;
	private final ByteBuffer tag;
	private final int errStatus;
	private final int errOff;
	private int next;
	private boolean referencePath; // past the engine's last good record: the reference decodes

	/** Decodes log[readerIndex, writerIndex) on the engine.  The log's readerIndex then advances
	 *  record by record as next() hands records out, as with SimpleDeterminantEncoder. */
	public EngineDecodedLog(ClonosEngine engine, ByteBuf log, DeterminantEncoder encoder) {
		this.log = log;
		this.encoder = encoder;
		this.base = log.readerIndex();
		final int len = log.readableBytes();
		final ByteBuf direct;
		if (log.isDirect() && log.nioBufferCount() == 1) {
			direct = log;
		} else {
			direct = Unpooled.directBuffer(Math.max(1, len)).writeBytes(log, base, len);
		}
		final int cap = len / 2 + 1; // a record is at least two bytes (OrderDeterminant)
		final int wcap = len / 6 + 1;
		this.recOff = ByteBuffer.allocateDirect(4 * cap).order(ByteOrder.nativeOrder());
		this.tag = ByteBuffer.allocateDirect(cap);
		final ByteBuffer v0 = ByteBuffer.allocateDirect(8 * cap);
		final ByteBuffer wIdx = ByteBuffer.allocateDirect(4 * wcap), wRc = ByteBuffer.allocateDirect(4 * wcap);
		final ByteBuffer wV1 = ByteBuffer.allocateDirect(8 * wcap), wVo = ByteBuffer.allocateDirect(4 * wcap);
		final ByteBuffer wVl = ByteBuffer.allocateDirect(4 * wcap), wSub = ByteBuffer.allocateDirect(wcap);
		final long[] res = new long[6];
		final ByteBuffer src = direct.nioBuffer(direct == log ? base : 0, len);
		final int st = nDecodeHost(engine.handle(), src, 0, len, recOff, tag, v0, wIdx, wRc, wV1, wVo, wVl, wSub, res);
		if (direct != log) {
			direct.release();
		}
		if (st != CLG_OK && res[2] == CLG_OK) {
			check(st); // engine failure, not a decode error
		}
		this.nRec = (int) res[0];
		this.errStatus = (int) res[2];
		this.errOff = (int) res[4];
	}

	/** Over a decode the engine already ran (replay-prep, EngineReplayPreparation): the
	 *  record offsets and tags of log[readerIndex, writerIndex), the record count and the first
	 *  error (status, offset; CLG_OK when none). */
	public EngineDecodedLog(ByteBuf log, DeterminantEncoder encoder, ByteBuffer recOff, ByteBuffer tag, int nRec,
							int errStatus, int errOff) {
		this.log = log;
		this.encoder = encoder;
		this.base = log.readerIndex();
		this.recOff = recOff;
		this.tag = tag;
		this.nRec = nRec;
		this.errStatus = errStatus;
		this.errOff = errOff;
	}

	/** decodeNext(ByteBuf, DeterminantPool) (:97-112): the next record, null at the end. */
	public Determinant next(DeterminantPool pool) {
		if (referencePath) {
			return encoder.decodeNext(log, pool);
		}
		if (next >= nRec) {
			if (errStatus == CLG_OK) {
				log.readerIndex(log.writerIndex());
				return null;
			}
			// the failing record: the reference decodes it (and everything after it)
			referencePath = true;
			log.readerIndex(base + errOff);
			return encoder.decodeNext(log, pool);
		}
		final int off = recOff.getInt(4 * next);
		final int t = tag.get(next);
		next++;
		log.readerIndex(base + off + 1); // past the tag: the per-type readers start at the fields
		final Determinant d;
		switch (t) {
			case Determinant.ORDER_DETERMINANT_TAG:
				d = encoder.decodeOrderDeterminant(log, pool.getOrderDeterminant());
				break;
			case Determinant.TIMESTAMP_DETERMINANT_TAG:
				d = encoder.decodeTimestampDeterminant(log, pool.getTimestampDeterminant());
				break;
			case Determinant.RNG_DETERMINANT_TAG:
				d = encoder.decodeRNGDeterminant(log, pool.getRNGDeterminant());
				break;
			case Determinant.BUFFER_BUILT_TAG:
				d = encoder.decodeBufferBuiltDeterminant(log, pool.getBufferBuiltDeterminant());
				break;
			case Determinant.TIMER_TRIGGER_DETERMINANT:
				d = encoder.decodeTimerTriggerDeterminant(log, pool.getTimerTriggerDeterminant());
				break;
			case Determinant.SOURCE_CHECKPOINT_DETERMINANT:
				d = encoder.decodeSourceCheckpointDeterminant(log, pool.getSourceCheckpointDeterminant());
				break;
			case Determinant.IGNORE_CHECKPOINT_DETERMINANT:
				d = encoder.decodeIgnoreCheckpointDeterminant(log, pool.getIgnoreCheckpointDeterminant());
				break;
			default: // SERIALIZABLE: the reference's ObjectInputStream path (the interface has no
				// per-type reader for it); the stream starts at the tag
				log.readerIndex(base + off);
				d = encoder.decodeNext(log, pool);
				break;
		}
		// the next record starts where the engine found it (identical to where the reader
		// stopped for every well-formed record)
		log.readerIndex(next < nRec ? base + recOff.getInt(4 * next) : (errStatus == CLG_OK ? log.writerIndex()
			: base + errOff));
		return d;
	}

	/** Records the engine decoded (before the first error, if any). */
	public int decodedRecords() {
		return nRec;
	}

	public boolean isReadable() {
		return referencePath ? log.isReadable() : (next < nRec || errStatus != CLG_OK);
	}
}
